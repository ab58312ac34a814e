#!/bin/bash
# Round 6 session 16: the partials' merge epilogue 8 columns a thread —
# parity (variant tests, realistic twins, C3 at size), in-process A/B on C3
# against the atomics (variant_part=0), one slice a row and the scalar merge,
# the C3 line with rocprofv3 kernel stats.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06s16
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_variant.py tests/test_gpu_realistic.py tests/test_gpu_fullsize.py \
    -m gpu -x -v --timeout 600 --timeout-method thread -k "not c4_full and not c5" -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/tests.log | head -20; exit $rc; }
AB_ENVS=";variant_part=0;variant_split=1;merge_rows8=0" AB_ROUNDS=4 timeout -k 10 400 python -u scripts/r06/ab_c3.py > $O/ab_c3.txt 2>&1 || { tail -20 $O/ab_c3.txt; exit 1; }
tail -4 $O/ab_c3.txt
timeout -k 10 600 python -u bench.py --config c3 --steps 50 --warmup 5 > $O/bench_c3.json 2> $O/bench_c3.err || exit 1
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('c3', d['ms_per_step'], d['value'], r.get('kernel_avg_ms'), (d.get('verified') or {}).get('ok'))" $O/bench_c3.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- \
    python3 bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline > $O/prof_c3.json 2> $O/prof_c3.err || exit $?
find $O -name "*kernel_trace.csv" -delete
