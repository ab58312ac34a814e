#!/bin/bash
# Round 4 session 22: the pinned staging upload (pack_overlap 3) parity and
# setup A/B; the SQ / TA pass of the 2 x 2 default sparse walk (VALU per 64
# products).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04s22
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 \
    --timeout-method thread -p no:cacheprovider -k "pack" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
AB_OUT=r04s22/abs bash scripts/r04/ab_setup.sh "" "--opt pack_overlap=3" || exit $?
A2="--steps 5 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD \
    SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv \
    -d $O/c2_sq -o run -- python3 bench.py $A2 > $O/c2_sq.json 2> $O/c2_sq.err &&
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_WAIT_ANY \
    SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD TA_TA_BUSY_sum --kernel-trace --output-format csv \
    -d $O/c2_lds -o run -- python3 bench.py $A2 > $O/c2_lds.json 2> $O/c2_lds.err &&
python3 scripts/pmc_sq_json.py $O/pmc_c2_sq.json c2 1000 sparse_tile_kernel $O/c2_sq $O/c2_lds
