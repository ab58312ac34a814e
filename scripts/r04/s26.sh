#!/bin/bash
# Round 4 session 26: parity of the 2 x 2 diagonal tiles (sparse_diag22) and
# the page-locked source upload; C2 A/B diag22 on/off; setup A/B page-locked
# (default) vs pageable caller buffers.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04s26
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_options.py -m gpu -x -v --timeout 120 \
    --timeout-method thread -p no:cacheprovider -k "sparse_complement_words_exact or option or pack" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
AB_OUT=r04s26/ab bash scripts/r04/ab.sh "--steps 20 --warmup 3" "--steps 20 --warmup 3 --opt sparse_diag22=0" || exit $?
AB_OUT=r04s26/abs bash scripts/r04/ab_setup.sh "" "--pageable" || exit $?
