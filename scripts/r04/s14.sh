#!/bin/bash
# Round 4 session 14: the fills' LDS-staged rare appends — parity of every
# fill route, the rare tiers and the variant tier; then the C2 and C3 lines
# (end to end) and the fill traces; the ring merge rework (edges, C5 line).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04s14
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_variant.py -m gpu -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider -k "sparse or rare_tier or fill_routes or variant or auto_method or sketch_merge_edges" \
    > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --opt trace=1 > $O/bench_c2.json 2> $O/bench_c2.err &&
timeout -k 10 300 python -u bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline --opt trace=1 > $O/bench_c3.json 2> $O/bench_c3.err &&
timeout -k 10 300 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err
rc=$?
for f in $O/bench_c2.json $O/bench_c3.json $O/bench_c5.json; do
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['ms_per_step'], d['value'], d['setup_s'], d['end_to_end']['seconds'], d['end_to_end']['pairs_per_s'])" $f
done
grep "fill\|bitsets:" $O/bench_c2.err $O/bench_c3.err | head -30
exit $rc
