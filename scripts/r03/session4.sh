#!/bin/bash
# Round-3 bench lines for the results table: C3 (METHOD_AUTO, full size)
# and the C4 per-rank slice, with rocprofv3 kernel stats of C3. Outputs under
# gpurun_out/r03/s4/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03/s4
mkdir -p $O
timeout -k 10 400 python -u bench.py --config c3 --steps 10 --warmup 2 > $O/bench_c3.json 2> $O/bench_c3.err &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- \
    python3 bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline > $O/prof_c3.json 2> $O/prof_c3.err &&
timeout -k 10 500 python -u bench.py --config c4 --rows 0:64 --force-exchange --steps 2 --warmup 1 \
    --opt trace=1 > $O/bench_c4_slice.json 2> $O/bench_c4_slice.err
rc=$?
for f in $O/bench_c3.json $O/bench_c4_slice.json; do
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['ms_per_step'], d['value'], d['roofline'].get('frac'), d['roofline'].get('kernel'))" $f
done
exit $rc
