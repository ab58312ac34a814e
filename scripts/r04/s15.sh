#!/bin/bash
# Round 4 session 15: C4 at its size on one GPU (tests/c4_worker.py: the
# consuming code all-gather on a one-rank RCCL communicator, METHOD_AUTO's
# variant-tier build from the gathered codes, rank 0's and the last rank's
# slices through the variant tier and the sorted join, three rows vs the
# oracle).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04s15
mkdir -p $O
rm -f gpurun_out/c4_worker.log
timeout -k 10 1050 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -q --timeout 1040 --timeout-method thread \
    -p no:cacheprovider -k c4_full > $O/c4test.log 2>&1
rc=$?
cp gpurun_out/c4_worker.log $O/ 2>/dev/null
tail -5 $O/c4test.log; cat $O/c4_worker.log
exit $rc
