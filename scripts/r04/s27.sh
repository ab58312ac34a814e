#!/bin/bash
# Round 4 session 27: parity of the pack's code-bits sort (pack_code_sort)
# and of the 2 x 4 micro-tiles (sparse_mt 4); setup A/B of the sort; C2 A/B
# 2 x 2 (default) vs 2 x 4.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04s27
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_options.py -m gpu -x -v --timeout 120 \
    --timeout-method thread -p no:cacheprovider -k "pack or option or k32 or sketch_build or sparse_complement_words_exact" \
    > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
AB_OUT=r04s27/ab bash scripts/r04/ab.sh "--steps 20 --warmup 3" "--steps 20 --warmup 3 --opt sparse_mt=4" || exit $?
AB_OUT=r04s27/abs bash scripts/r04/ab_setup.sh "" "--opt pack_code_sort=0" || exit $?
timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 3 --warmup 1 --opt trace=1 > $O/c2_trace.json 2> $O/c2_trace.err
