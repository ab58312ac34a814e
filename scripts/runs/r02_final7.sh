#!/bin/bash
# Round-2 closing measurement of the default path after the pack rework: every -m gpu test, smoke, rocprofv3 stats,
# FETCH/WRITE PMC -> profiles/pmc_c2.json, the default bench line
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/final7
mkdir -p $D
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > $D/gputest.log 2>&1 || { tail -40 $D/gputest.log; exit 1; }
tail -1 $D/gputest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
A="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline"
K="sparse_tile_kernel5<3, 8, 1, 2, false>"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- $A > $D/trace.json 2> $D/trace.log || exit 1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $D/fetch -o run -- $A > $D/fetch.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $D/write -o run -- $A > $D/write.log 2>&1 || exit 1
python3 scripts/pmc_json.py $D/fetch $D/write "$K" profiles/pmc_c2.json c2 1000 && cp profiles/pmc_c2.json $D/ || exit 1
timeout -k 10 500 python bench.py > $D/bench_default.json 2> $D/bench_default.err || { tail -20 $D/bench_default.err; exit 1; }
cat $D/bench_default.json
