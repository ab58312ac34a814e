#!/bin/bash
# SQ counter passes for the sketch kernels (AB_VARIANTS picks the options) (counters only, no trace domains).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AB_ROUNDS=1 AB_N=${AB_N:-10000} AB_VARIANTS=${AB_VARIANTS:-default}
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE \
   --kernel-trace --output-format csv -d gpurun_out/pmc_sk1 -o run -- python3 scripts/ab_sketch.py > gpurun_out/pmc_sk1.log 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INST_LEVEL_LDS \
   --kernel-trace --output-format csv -d gpurun_out/pmc_sk2 -o run -- python3 scripts/ab_sketch.py > gpurun_out/pmc_sk2.log 2>&1
