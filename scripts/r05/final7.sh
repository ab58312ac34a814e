#!/bin/bash
# round 5 final (seventh pass: the final tree): the whole -m gpu suite, smoke(), then every
# config's line on the final kernels (C2 and C3 also under rocprofv3
# --kernel-trace --stats; C2-realistic's kernel stats)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05final7
mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread -p no:cacheprovider \
    > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/smoke.log 2>&1 || exit $?
tail -2 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- \
    python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_c2_prof.json 2> $O/bench_c2_prof.err || exit $?
timeout -k 10 400 python -u bench.py --config c3 --steps 50 --warmup 5 > $O/bench_c3.json 2> $O/bench_c3.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- \
    python3 bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline > $O/prof_c3.json 2> $O/prof_c3.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2r -o run -- \
    python3 bench.py --config c2r --steps 20 --warmup 3 > $O/bench_c2r.json 2> $O/bench_c2r.err || exit $?
timeout -k 10 500 python -u bench.py --config c4 --rows 0:1024 --force-exchange --steps 10 --warmup 3 --opt split_build=8 \
    --opt trace=1 > $O/bench_c4_slice1024.json 2> $O/bench_c4_slice1024.err || exit $?
grep -E "gdist: (variant|bitsets|fill|postings|range|build)" $O/bench_c4_slice1024.err > $O/c4_build_trace.txt
find $O -name "*kernel_trace.csv" -delete
for f in bench_c2 bench_c3 bench_c2r bench_c4_slice1024; do
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1].split('/')[-1], d['ms_per_step'], d['value'], r.get('kernel_avg_ms'), r.get('frac'), r.get('traffic'), r.get('step_kernel_span_ms'), (d.get('cpu_baseline') or {}).get('value'), (d.get('end_to_end') or {}).get('seconds'))" $O/$f.json
done
