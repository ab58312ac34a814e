#!/bin/bash
# Round 6 session 19: the sketch ring kernel's 4-step rounds (one LDS round
# trip per four merge steps, option sketch_quad) — sketch parity (every
# merge loop, C5 at size under sketch_quad=1 too), in-process A/B on C5.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06s19
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -v --timeout 500 \
    --timeout-method thread -k "sketch or c5" -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/tests.log | head -20; exit $rc; }
AB_VARIANTS="default,sketch_quad=1,sketch_quad=1+sketch_cap=200,sketch_quad=1+sketch_cap=240" AB_ROUNDS=3 \
    timeout -k 10 700 python -u scripts/ab_sketch.py > $O/ab_c5.txt 2>&1 || { tail -20 $O/ab_c5.txt; exit 1; }
tail -6 $O/ab_c5.txt
