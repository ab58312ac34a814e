#!/bin/bash
# Round 6 session 22: the C4 variant walk with two members a lane a step
# (option variant_w2) — variant parity (poisoned replays, column chunks),
# in-process A/B on the C4 slice, and the C4-realistic slice line with it.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06s22
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_variant.py -m gpu -x -v --timeout 500 --timeout-method thread \
    -k "poisoned or column_chunks or variant_tier" -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/tests.log | head -20; exit $rc; }
AB_ENVS=";variant_w2=1" AB_ROUNDS=3 timeout -k 10 600 python -u scripts/r05/ab_c4.py > $O/ab_c4.txt 2>&1 || { tail -20 $O/ab_c4.txt; exit 1; }
tail -2 $O/ab_c4.txt
