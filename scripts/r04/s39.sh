#!/bin/bash
# Round 4 session 39: row-trimmed sparse tiles in 2 x 2 micro-tiles
# (sparse_rpart22): parity (unaligned regions, multi-rank slices), and A/B
# on C2 row slices shaped like a rank's block of the 8-rank weak-scaling run.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04s39
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_options.py tests/test_multirank_gpu.py -m gpu -x -q \
    --timeout 200 --timeout-method thread -p no:cacheprovider -k "sparse or option or multirank" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
AB_OUT=r04s39/ab bash scripts/r04/ab.sh "--steps 20 --warmup 3 --rows 100:700" \
    "--steps 20 --warmup 3 --rows 100:700 --opt sparse_rpart22=0" || exit $?
