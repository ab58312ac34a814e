#!/bin/bash
# Round 6 final evidence, part 2 (the final tree): every other config's line
# (C2-realistic, C3 and C3-realistic with rocprofv3 kernel stats, the C4 and
# C4-realistic per-rank slices, C5).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06final2
mkdir -p $O
line() {   # name, bench args
    local name=$1; shift
    timeout -k 10 600 python -u bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo "line $name failed"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1].split('/')[-1], d['ms_per_step'], d['value'], r.get('kernel_avg_ms'), r.get('frac'), r.get('traffic'), (d.get('cpu_baseline') or {}).get('value'), (d.get('verified') or {}).get('ok'))" $O/$name.json
}
line bench_c2r --config c2r --steps 20 --warmup 3
line bench_c3 --config c3 --steps 50 --warmup 5
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- \
    python3 bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline > $O/prof_c3.json 2> $O/prof_c3.err || exit $?
line bench_c3r --config c3r --steps 50 --warmup 5
line bench_c4_slice1024 --config c4 --rows 0:1024 --force-exchange --steps 10 --warmup 3 --opt split_build=8
line bench_c4r_slice1024 --config c4r --rows 0:1024 --force-exchange --steps 10 --warmup 3 --opt split_build=8
line bench_c5 --config c5 --steps 3 --warmup 1
find $O -name "*kernel_trace.csv" -delete
