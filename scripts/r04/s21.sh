#!/bin/bash
# Round 4 session 21: parity of the workgroup merge fill (fill_sort default /
# 5) and the 2 x 2 micro-tiles (sparse_mt 2), then C2 A/B of the walk shapes
# and the fill's setup A/B, and a C2 stage trace.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04s21
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_options.py -m gpu -x -v --timeout 120 \
    --timeout-method thread -p no:cacheprovider -k "sparse_complement_words_exact or fill or all_ones or option" \
    > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
AB_OUT=r04s21/ab bash scripts/r04/ab.sh "--steps 20 --warmup 3" "--steps 20 --warmup 3 --opt sparse_mt=2 --opt sparse_sun=3" \
    "--steps 20 --warmup 3 --opt sparse_mt=2 --opt sparse_sun=2" "--steps 20 --warmup 3 --opt sparse_mt=2" || exit $?
AB_OUT=r04s21/abs bash scripts/r04/ab_setup.sh "" "--opt fill_sort=5" || exit $?
timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 3 --warmup 1 --opt trace=1 > $O/c2_trace.json 2> $O/c2_trace.err
