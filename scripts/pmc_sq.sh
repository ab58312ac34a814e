#!/bin/bash
# SQ counter pass for the bitset kernel A/B (counters only, no trace domains).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AB_ROUNDS=${AB_ROUNDS:-2}
mkdir -p gpurun_out
rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE \
   --kernel-trace --output-format csv -d gpurun_out/pmc_sq -o run -- python3 scripts/ab_bitset.py > gpurun_out/pmc_sq.log 2>&1
