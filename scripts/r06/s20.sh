#!/bin/bash
# Round 6 session 20: the sketch ring kernel in 64 x 64 tiles, four pairs a
# thread stepped together (option sketch_tile64) — sketch parity (every
# merge loop incl. the new one), in-process A/B on C5 (identical counts on
# 2,048 rows checked), the C5 line with it.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06s20
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 \
    --timeout-method thread -k "sketch" -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/tests.log | head -20; exit $rc; }
AB_VARIANTS="default,sketch_tile64=1,sketch_tile64=1+sketch_cap=200" AB_ROUNDS=3 \
    timeout -k 10 700 python -u scripts/ab_sketch.py > $O/ab_c5.txt 2>&1 || { tail -20 $O/ab_c5.txt; exit 1; }
tail -8 $O/ab_c5.txt
