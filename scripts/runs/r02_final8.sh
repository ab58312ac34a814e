#!/bin/bash
# After pack_chunk 2^28 became the default: every -m gpu test, smoke, the default bench line
set -o pipefail
D=gpurun_out/final8
mkdir -p $D
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > $D/gputest.log 2>&1 || { tail -40 $D/gputest.log; exit 1; }
tail -1 $D/gputest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 500 python bench.py > $D/bench_default.json 2> $D/bench_default.err || { tail -20 $D/bench_default.err; exit 1; }
cat $D/bench_default.json
