#!/bin/bash
# round 5 session 10: sparse chunk counts below the 1,023-word cap (the
# complement-bit bound decides exactness) on C2 and C2-realistic, and the
# C2-realistic step's kernels under rocprofv3
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05s10
mkdir -p $O
AB_ROUNDS=5 AB_ENVS=";sparse_chunks=24;sparse_chunks=31;sparse_chunks=40;sparse_chunks=48" \
    timeout -k 10 300 python -u scripts/ab_env.py > $O/ab_c2.txt 2> $O/ab_c2.err || exit $?
cat $O/ab_c2.txt
AB_CONFIG=c2r AB_ROUNDS=5 AB_ENVS=";sparse_chunks=29;sparse_chunks=40;sparse_chunks=50;sparse_chunks=62" \
    timeout -k 10 400 python -u scripts/ab_env.py > $O/ab_c2r.txt 2> $O/ab_c2r.err || exit $?
cat $O/ab_c2r.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2r -o run -- \
    python3 bench.py --config c2r --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_c2r.json 2> $O/bench_c2r.err || exit $?
find $O/prof_c2r -name "*kernel_trace.csv" -delete
python3 - <<'PY'
import csv, glob
for f in glob.glob('gpurun_out/r05s10/prof_c2r/**/*kernel_stats.csv', recursive=True):
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: -float(r['TotalDurationNs']))
    for r in rows[:12]:
        print(r['Name'][:60], r['Calls'], round(float(r['AverageNs']) / 1e3, 1), 'us avg')
PY
