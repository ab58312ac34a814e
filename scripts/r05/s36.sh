#!/bin/bash
# round 5 session 36: the sparse chunk reduce's loads issued in one batch;
# the variant split default: parity (sparse, variant), C2 / C2r / C4 lines
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05s36
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_variant.py tests/test_gpu_options.py tests/test_gpu_realistic.py -m gpu -x -q --timeout 600 \
    --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- \
    python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/c2_prof.json 2> $O/c2_prof.err || exit $?
find $O -name "*kernel_trace.csv" -delete
grep -E "sparse_tile|sparse_reduce" $O/prof_c2/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-140
timeout -k 10 300 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err || exit $?
timeout -k 10 400 python -u bench.py --config c2r --steps 20 --warmup 3 > $O/bench_c2r.json 2> $O/bench_c2r.err || exit $?
timeout -k 10 500 python -u bench.py --config c4 --rows 0:1024 --force-exchange --steps 10 --warmup 3 --opt split_build=8 \
    > $O/bench_c4_slice1024.json 2> $O/bench_c4_slice1024.err || exit $?
for f in bench_c2 bench_c2r bench_c4_slice1024; do
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1].split('/')[-1], d['ms_per_step'], d['value'], r.get('kernel_avg_ms'), r.get('frac'), r.get('step_kernel_span_ms'), (d.get('cpu_baseline') or {}).get('value'))" $O/$f.json
done
