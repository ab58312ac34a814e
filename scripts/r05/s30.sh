#!/bin/bash
# round 5 session 30: the C4 variant wave walk with 128 KiB of 16-bit
# counters (65,536 columns a chunk: 2 chunks instead of 4)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05s30
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_variant.py tests/test_gpu_options.py -m gpu -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider -k "column_chunks or option" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
AB_ENVS=";variant_wide=1" timeout -k 10 500 python -u scripts/r05/ab_c4.py > $O/ab_c4.txt 2> $O/ab_c4.err || exit $?
grep -E "built|^\[|mismatch|equal" $O/ab_c4.txt
