#!/bin/bash
# Round 4 session 40 (the final tree): the whole -m gpu suite as
# the driver runs it, then smoke().
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04s40
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
    -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
rc=$?; tail -3 $O/smoke.log; exit $rc
