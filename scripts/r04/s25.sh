#!/bin/bash
# Round 4 session 25: the two-thread upload (pack_overlap 3) parity and setup A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04s25
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 \
    --timeout-method thread -p no:cacheprovider -k "pack" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
AB_OUT=r04s25/abs bash scripts/r04/ab_setup.sh "" "--opt pack_overlap=3" || exit $?
