#!/bin/bash
# Ring sketch kernel as the default: the whole -m gpu suite, smoke, the C2
# and C5 bench lines, rocprofv3 kernel trace + stats of the C5 line, and the
# ring kernel's SQ/LDS counters (10,000 sketches). Outputs under gpurun_out/r03s8/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03s8
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider \
    --durations=25 > $O/gputest.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $O/bench_c2.json 2> $O/bench_c2.err &&
timeout -k 10 400 python -u bench.py --config c5 --steps 3 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o run -- \
    python3 bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > $O/prof_c5.json 2> $O/prof_c5.err &&
AB_VARIANTS=default bash scripts/pmc_sketch.sh &&
python3 scripts/pmc_summary.py gpurun_out/pmc_sk1 gpurun_out/pmc_sk2 --kernel sketch_ring > $O/pmc_ring.txt
rc=$?
tail -3 $O/gputest.log; cat $O/smoke.log
cut -c1-400 $O/bench_c2.json $O/bench_c5.json
cat $O/pmc_ring.txt
exit $rc
