#!/bin/bash
# round 5 final lines (C3, C2-realistic, C5) on the final kernels, C3 also
# under rocprofv3 --kernel-trace --stats; a last C3 issue-order A/B first
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05final4
mkdir -p $O
for o in "--opt dense_first=0" ""; do
  timeout -k 10 300 python -u bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline $o > $O/c3ab.json 2> $O/c3ab.err || exit $?
  python3 -c "
import json; d=json.load(open('$O/c3ab.json')); r=d['roofline']
print('c3 [$o]', d['ms_per_step'], r['kernel_avg_ms'], [o['kernel_avg_ms'] for o in r.get('other', [])], d['verified']['ok'])"
done
timeout -k 10 400 python -u bench.py --config c3 --steps 50 --warmup 5 > $O/bench_c3.json 2> $O/bench_c3.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- \
    python3 bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline > $O/prof_c3.json 2> $O/prof_c3.err || exit $?
find $O/prof_c3 -name "*kernel_trace.csv" -delete
timeout -k 10 400 python -u bench.py --config c2r --steps 20 --warmup 3 > $O/bench_c2r.json 2> $O/bench_c2r.err || exit $?
timeout -k 10 500 python -u bench.py --config c5 --steps 3 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err || exit $?
for f in bench_c3 bench_c2r bench_c5; do
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1].split('/')[-1], d['ms_per_step'], d['value'], r.get('kernel_avg_ms'), r.get('frac'), r.get('traffic'), (d.get('cpu_baseline') or {}).get('value'), (d.get('end_to_end') or {}).get('seconds'), d['verified'])" $O/$f.json
done
