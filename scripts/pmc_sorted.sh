#!/bin/bash
# SQ counter passes for the sorted join kernels (counters only, no trace domains).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ARGS=${BENCH_ARGS:-"--config c3 --method sorted --n 3000 --steps 1 --warmup 0 --no-cpu-baseline"}
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE \
   --kernel-trace --output-format csv -d gpurun_out/pmc_so1 -o run -- python3 bench.py $ARGS > gpurun_out/pmc_so1.log 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU \
   --kernel-trace --output-format csv -d gpurun_out/pmc_so2 -o run -- python3 bench.py $ARGS > gpurun_out/pmc_so2.log 2>&1
