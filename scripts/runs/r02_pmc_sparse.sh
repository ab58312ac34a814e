#!/bin/bash
# PMC passes of the sparse tile kernels v1 / v2 on C2 (counters only, one pass per run)
set -o pipefail
export TMPDIR=/tmp
for v in 1 2; do
  A="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --opt sparse_kernel=$v"
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD --kernel-trace --output-format csv -d gpurun_out/pm$v/a -o run -- $A > gpurun_out/pm$v.a.log 2>&1 || exit 1
  timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INST_LEVEL_VMEM --kernel-trace --output-format csv -d gpurun_out/pm$v/b -o run -- $A > gpurun_out/pm$v.b.log 2>&1 || exit 1
  timeout -s KILL 150 rocprofv3 --pmc TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pm$v/c -o run -- $A > gpurun_out/pm$v.c.log 2>&1 || exit 1
  python3 scripts/pmc_summary.py gpurun_out/pm$v --kernel sparse_tile > gpurun_out/pm$v.txt
done
cat gpurun_out/pm1.txt gpurun_out/pm2.txt
