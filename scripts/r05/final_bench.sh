#!/bin/bash
# round 5 final B: the bench lines of every config on the final tree, the
# default (C2) line also under rocprofv3 --kernel-trace --stats
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05final
mkdir -p $O
timeout -k 10 300 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- \
    python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_c2_prof.json 2> $O/bench_c2_prof.err || exit $?
find $O/prof_c2 -name "*kernel_trace.csv" -delete
timeout -k 10 400 python -u bench.py --config c2r --steps 10 --warmup 2 > $O/bench_c2r.json 2> $O/bench_c2r.err || exit $?
timeout -k 10 300 python -u bench.py --config c3 --steps 10 --warmup 2 > $O/bench_c3.json 2> $O/bench_c3.err || exit $?
timeout -k 10 500 python -u bench.py --config c4 --rows 0:1024 --force-exchange --steps 5 --warmup 1 --opt split_build=8 \
    > $O/bench_c4_slice1024.json 2> $O/bench_c4_slice1024.err || exit $?
timeout -k 10 400 python -u bench.py --config c5 --steps 3 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err || exit $?
for f in bench_c2 bench_c2r bench_c3 bench_c4_slice1024 bench_c5; do
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1].split('/')[-1], d['ms_per_step'], d['value'], r.get('kernel_avg_ms'), r.get('frac'), r.get('traffic'), (d.get('cpu_baseline') or {}).get('value'), (d.get('end_to_end') or {}).get('seconds'))" $O/$f.json
done
