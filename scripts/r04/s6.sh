#!/bin/bash
# Round 4 session 6: the variant tier's parity tests first, then the session-5
# evidence (suite, smoke, C2/C3 lines, C3 PMC, FETCH calibration, C4 at size).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04s6
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_variant.py -m gpu -x -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $O/variant.log 2>&1
rc=$?
tail -12 $O/variant.log
exit $rc
