#!/bin/bash
# round 5 session 18: greedy representatives of a gathered collection with
# the columns sharded over the ranks (2 and 3 host-transport ranks), and the
# single-GPU reps tests
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05s18
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_multirank_gpu.py tests/test_gpu_parity.py tests/test_gpu_variant.py tests/test_gpu_options.py \
    -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider -k "multirank or reps or option" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
