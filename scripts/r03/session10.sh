#!/bin/bash
# Round-end evidence with the final code: the whole -m gpu suite, smoke, every
# config's bench line (C2, C2-realistic, C3 with rocprofv3 stats, C5, the C4
# per-rank slice through the code all-gather on a one-rank RCCL
# communicator), and a short sketch steps-per-phase A/B. Outputs under
# gpurun_out/r03s10/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03s10
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider \
    --durations=25 > $O/gputest.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $O/bench_c2.json 2> $O/bench_c2.err &&
timeout -k 10 300 python -u bench.py --config c2r --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_c2r.json 2> $O/bench_c2r.err &&
timeout -k 10 400 python -u bench.py --config c3 --steps 10 --warmup 2 > $O/bench_c3.json 2> $O/bench_c3.err &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- \
    python3 bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline > $O/prof_c3.json 2> $O/prof_c3.err &&
timeout -k 10 400 python -u bench.py --config c5 --steps 3 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err &&
AB_ROUNDS=1 AB_VARIANTS=default,sketch_cap=200,sketch_cap=240 timeout -k 10 400 \
    python -u scripts/ab_sketch.py > $O/ab_c5_cap.txt 2>&1 &&
timeout -k 10 600 python -u bench.py --config c4 --rows 0:64 --force-exchange --steps 2 --warmup 1 \
    --opt trace=1 > $O/bench_c4_slice.json 2> $O/bench_c4_slice.err
rc=$?
tail -3 $O/gputest.log; cat $O/smoke.log $O/ab_c5_cap.txt
for f in $O/bench_c2.json $O/bench_c2r.json $O/bench_c3.json $O/bench_c5.json $O/bench_c4_slice.json; do
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['ms_per_step'], d['value'], d['roofline'].get('frac'), d['roofline'].get('kernel'))" $f
done
exit $rc
