#!/bin/bash
# One GPU call after the group tier: the parity suite, smoke, the C2 and
# C2-realistic bench lines (each step under its own time limit, stopping at
# the first failure). Outputs under gpurun_out/r03/s2/.
set -o pipefail
O=gpurun_out/r03/s2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider \
    --durations=20 > $O/gputest.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $O/bench_c2.json 2> $O/bench_c2.err &&
timeout -k 10 300 python -u bench.py --config c2r --steps 20 --warmup 3 > $O/bench_c2r.json 2> $O/bench_c2r.err
rc=$?
tail -3 $O/gputest.log
cat $O/bench_c2.json $O/bench_c2r.json 2>/dev/null | cut -c1-300
exit $rc
