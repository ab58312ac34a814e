#!/bin/bash
# Round 4 session 23: parity of the claimed word batches (sparse_dyn) and
# the C2 A/B: claimed batches vs equal runs, chunk counts, rare rows apart
# (the tile workgroups' own time).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04s23
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_options.py -m gpu -x -v --timeout 120 \
    --timeout-method thread -p no:cacheprovider -k "sparse_complement_words_exact or option" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
AB_OUT=r04s23/ab bash scripts/r04/ab.sh "--steps 20 --warmup 3" "--steps 20 --warmup 3 --opt sparse_dyn=0" \
    "--steps 20 --warmup 3 --opt sparse_chunks=93" "--steps 20 --warmup 3 --opt sparse_chunks=124" \
    "--steps 20 --warmup 3 --opt sparse_rare=0" || exit $?
