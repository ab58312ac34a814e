#!/bin/bash
# round 5 final A: the whole -m gpu suite and smoke() on the final tree
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05final
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider \
    > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/smoke.log 2>&1 || exit $?
tail -2 $O/smoke.log
