#!/bin/bash
# Round 6 session 4: the whole -m gpu suite with durations (VERDICT r5 item
# 6: well inside the 900 s step), smoke(), the C2 line and its rocprofv3
# kernel stats, C3 and its realistic twin, the C4 slice (the MFMA tiles now
# read a chunk's fragments one chunk ahead).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06s4
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=40 \
    -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/smoke.log 2>&1 || exit $?
tail -2 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- \
    python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_c2_prof.json 2> $O/bench_c2_prof.err || exit $?
timeout -k 10 400 python -u bench.py --config c3 --steps 50 --warmup 5 > $O/bench_c3.json 2> $O/bench_c3.err || exit $?
timeout -k 10 400 python -u bench.py --config c3r --steps 50 --warmup 5 > $O/bench_c3r.json 2> $O/bench_c3r.err || exit $?
timeout -k 10 500 python -u bench.py --config c4 --rows 0:1024 --force-exchange --steps 10 --warmup 3 --opt split_build=8 \
    > $O/bench_c4_slice1024.json 2> $O/bench_c4_slice1024.err || exit $?
find $O -name "*kernel_trace.csv" -delete
for f in bench_c2 bench_c3 bench_c3r bench_c4_slice1024; do
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1].split('/')[-1], d['ms_per_step'], d['value'], r.get('kernel_avg_ms'), r.get('frac'), r.get('traffic'), (d.get('cpu_baseline') or {}).get('value'), d.get('verified'))" $O/$f.json
done
