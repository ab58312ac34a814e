#!/bin/bash
# Round 6 session 7: keyless variant kmers routed to the rare tier (parity:
# variant tier modes, split build, realistic twins), the epilogue A/B on C3
# (four columns a thread over ~1,024 looping block rows vs one column a
# thread), and the C4 / C4-realistic slices.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06s7
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_variant.py tests/test_gpu_realistic.py tests/test_gpu_parity.py::test_distance_epilogue_modes \
    > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
line() {   # name, bench args
    local name=$1; shift
    timeout -k 10 600 python -u bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo "line $name failed"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1].split('/')[-1], d['ms_per_step'], d['value'], r.get('kernel_avg_ms'), r.get('frac'), r.get('traffic'), (d.get('cpu_baseline') or {}).get('value'), (d.get('verified') or {}).get('ok'))" $O/$name.json
}
for r in 1 2; do
  line c3_epi2_$r --config c3 --steps 50 --warmup 5 --no-cpu-baseline
  line c3_epi1_$r --config c3 --steps 50 --warmup 5 --no-cpu-baseline --opt epilogue_rows=1
done
line bench_c4r_slice1024 --config c4r --rows 0:1024 --force-exchange --steps 10 --warmup 3 --opt split_build=8 --opt trace=1
grep -E "keyless|variant tier:" $O/bench_c4r_slice1024.err | head -5
line bench_c4_slice1024 --config c4 --rows 0:1024 --force-exchange --steps 10 --warmup 3 --opt split_build=8 --opt trace=1
grep -E "keyless|variant tier:" $O/bench_c4_slice1024.err | head -5
