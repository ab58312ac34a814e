#!/bin/bash
# Round 4 session 33: parity of the batch-bound prefetch (sparse_prefetch)
# and the C2 A/B against the default walk.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04s33
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_options.py -m gpu -x -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider -k "sparse_complement_words_exact or option" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
AB_OUT=r04s33/ab bash scripts/r04/ab.sh "--steps 20 --warmup 3" "--steps 20 --warmup 3 --opt sparse_prefetch=1" \
    "--steps 20 --warmup 3 --opt sparse_prefetch=1 --opt sparse_sun=2" || exit $?
