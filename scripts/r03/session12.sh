#!/bin/bash
# Closing check of the round's final tree: the whole -m gpu suite, smoke
# (bitset + sorted + sketch ring paths against the oracle), the default bench
# line. Outputs under gpurun_out/r03s12/.
set -o pipefail
O=gpurun_out/r03s12
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider \
    --durations=25 > $O/gputest.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err
rc=$?
tail -3 $O/gputest.log; cat $O/smoke.log; cut -c1-300 $O/bench_c2.json
exit $rc
