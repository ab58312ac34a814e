#!/bin/bash
# round 5 session 10: sparse chunk counts below the 1,023-word cap on C2 (the
# complement-bit bound decides exactness), C3's rare threshold against the
# matrix-core dense rate, and the C2-realistic step's kernels under rocprofv3
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05s10
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_variant.py tests/test_gpu_options.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 -k "variant or option or rare" \
    --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
AB_ENVS=";variant_cores=1" timeout -k 10 400 python -u scripts/r05/ab_c4.py > $O/ab_c4.txt 2> $O/ab_c4.err || exit $?
grep -E "built|^\[" $O/ab_c4.txt
AB_ROUNDS=5 AB_ENVS=";sparse_chunks=24;sparse_chunks=31;sparse_chunks=40;sparse_chunks=48" \
    timeout -k 10 300 python -u scripts/ab_env.py > $O/ab_c2.txt 2> $O/ab_c2.err || exit $?
cat $O/ab_c2.txt
timeout -k 10 300 python -u bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline --opt serial_step=1 > $O/c3_serial.json 2> $O/c3_serial.err || exit $?
timeout -k 10 300 python -u bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline > $O/c3.json 2> $O/c3.err || exit $?
python3 -c "
import json
for f in ('c3_serial', 'c3'):
    d=json.load(open('$O/%s.json' % f)); r=d['roofline']; print(f, d['ms_per_step'], r['kernel'][:20], r['kernel_avg_ms'], [(o['kernel'][:20], o['kernel_avg_ms']) for o in r.get('other', [])])"
for t in 20 28 31; do
  timeout -k 10 300 python -u bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline --opt rare_t=$t \
      > $O/c3_t$t.json 2> $O/c3_t$t.err || exit $?
  python3 -c "import json; d=json.load(open('$O/c3_t$t.json')); r=d['roofline']; c=d['config']; print('c3 T=$t', d['ms_per_step'], c['bitset_words_per_set'], c['rare_tier'], r['kernel_avg_ms'], [(o['kernel'][:20], o['kernel_avg_ms']) for o in r.get('other', [])])"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2r -o run -- \
    python3 bench.py --config c2r --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_c2r.json 2> $O/bench_c2r.err || exit $?
find $O/prof_c2r -name "*kernel_trace.csv" -delete
python3 - <<'PY'
import csv, glob, json
d = json.load(open('gpurun_out/r05s10/bench_c2r.json'))
print('c2r', d['ms_per_step'], d['config']['complement_sparse'])
for f in glob.glob('gpurun_out/r05s10/prof_c2r/**/*kernel_stats.csv', recursive=True):
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: -float(r['TotalDurationNs']))
    for r in rows[:12]:
        print(r['Name'][:60], r['Calls'], round(float(r['AverageNs']) / 1e3, 1), 'us avg')
PY
