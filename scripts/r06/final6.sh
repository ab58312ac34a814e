#!/bin/bash
# Round 6 final evidence, part 6 (the final tree, after the walks' slice
# defaults: C3's short walk one slice a row, the C4 variant walk ~64 slices a
# CU): the whole -m gpu suite, smoke(), the C3 / C3r / C4 / C4r lines (C3
# also under rocprofv3 kernel stats).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06final6
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=20 \
    -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/tests.log | head -20; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/smoke.log 2>&1 || exit $?
tail -2 $O/smoke.log
line() {   # name, bench args
    local name=$1; shift
    timeout -k 10 600 python -u bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo "line $name failed"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1].split('/')[-1], d['ms_per_step'], d['value'], r.get('kernel_avg_ms'), r.get('frac'), r.get('traffic'), (d.get('cpu_baseline') or {}).get('value'), (d.get('verified') or {}).get('ok'))" $O/$name.json
}
line bench_c3 --config c3 --steps 50 --warmup 5
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- \
    python3 bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline > $O/prof_c3.json 2> $O/prof_c3.err || exit $?
line bench_c3r --config c3r --steps 50 --warmup 5
line bench_c4_slice1024 --config c4 --rows 0:1024 --force-exchange --steps 10 --warmup 3 --opt split_build=8
line bench_c4r_slice1024 --config c4r --rows 0:1024 --force-exchange --steps 10 --warmup 3 --opt split_build=8
find $O -name "*kernel_trace.csv" -delete
