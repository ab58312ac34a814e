#!/bin/bash
# round 5 session 17: the variant walk with two entries a wave in flight
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05s17
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_variant.py tests/test_gpu_options.py -m gpu -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
AB_ENVS=";variant_pair=1" AB_ROUNDS=4 timeout -k 10 400 python -u scripts/r05/ab_c4.py > $O/ab_c4.txt 2> $O/ab_c4.err || exit $?
grep -E "built|^\[" $O/ab_c4.txt
