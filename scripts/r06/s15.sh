#!/bin/bash
# Round 6 session 15: the short walk's partial rows (stored, merged by the
# step's epilogue) with the MFMA tiles storing every pair — parity (variant,
# realistic twins, C3 at size, MFMA tiles), then in-process A/B against the
# atomics (variant_part=0) on C3 and C3r, and the C3 / C3r lines.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06s15
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_variant.py tests/test_gpu_realistic.py tests/test_gpu_fullsize.py \
    -m gpu -x -v --timeout 600 --timeout-method thread -k "not c4_full and not c5" -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/tests.log | head -20; exit $rc; }
AB_ENVS=";variant_part=0" AB_ROUNDS=4 timeout -k 10 400 python -u scripts/r06/ab_c3.py > $O/ab_c3.txt 2>&1 || { tail -20 $O/ab_c3.txt; exit 1; }
tail -2 $O/ab_c3.txt
AB_CONFIG=c3r AB_ENVS=";variant_part=0" AB_ROUNDS=3 timeout -k 10 400 python -u scripts/r06/ab_c3.py > $O/ab_c3r.txt 2>&1 || { tail -20 $O/ab_c3r.txt; exit 1; }
tail -2 $O/ab_c3r.txt
line() {   # name, bench args
    local name=$1; shift
    timeout -k 10 600 python -u bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo "line $name failed"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1].split('/')[-1], d['ms_per_step'], d['value'], r.get('kernel')[:40], r.get('kernel_avg_ms'), r.get('frac'), [(o.get('kernel','')[:30], o.get('kernel_avg_ms'), o.get('frac')) for o in r.get('other') or []], (d.get('verified') or {}).get('ok'))" $O/$name.json
}
line bench_c3 --config c3 --steps 50 --warmup 5
line bench_c3r --config c3r --steps 50 --warmup 5
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- \
    python3 bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline > $O/prof_c3.json 2> $O/prof_c3.err || exit $?
find $O -name "*kernel_trace.csv" -delete
