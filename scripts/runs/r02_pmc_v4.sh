#!/bin/bash
# PMC of sparse v4 (grid walk from LDS) vs v1 on C2
set -o pipefail
export TMPDIR=/tmp
for v in 4 1; do
  A="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --opt sparse_kernel=$v --opt sparse_sun=1"
  [ $v = 1 ] && A="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --opt sparse_kernel=1"
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU --kernel-trace --output-format csv -d gpurun_out/q$v/a -o run -- $A > gpurun_out/q$v.a.log 2>&1 || exit 1
  timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_ADDR_CONFLICT SQ_INSTS_VMEM_RD --kernel-trace --output-format csv -d gpurun_out/q$v/b -o run -- $A > gpurun_out/q$v.b.log 2>&1 || exit 1
  timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_INSTS_SMEM --kernel-trace --output-format csv -d gpurun_out/q$v/c -o run -- $A > gpurun_out/q$v.c.log 2>&1 || true
  python3 scripts/pmc_summary.py gpurun_out/q$v --kernel sparse_tile > gpurun_out/q$v.txt
done
paste gpurun_out/q4.txt gpurun_out/q1.txt | awk '{print $2, $4, $8}'
