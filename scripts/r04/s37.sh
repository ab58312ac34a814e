#!/bin/bash
# Round 4 session 37: the collection's last partial row block walked without
# row trimming (2 x 2 / diagonal 2 x 2): sparse parity and C2 lines.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04s37
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_realistic.py -m gpu -x -q --timeout 200 \
    --timeout-method thread -p no:cacheprovider -k "sparse or realistic or group" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
AB_OUT=r04s37/ab bash scripts/r04/ab.sh "--steps 20 --warmup 3" || exit $?
