#!/bin/bash
# Round 4 session 11: the reworked sparse walk (mbcnt word lookup, packed
# reciprocal, virtual word) — sparse parity first; then the C2 line with a
# rocprofv3 summary; the flattened rare row walk (C3 A/B); the variant tier's tests.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04s11
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider -k "sparse or graph_replay or rare_tier or fill_routes" > $O/sparse.log 2>&1
rc=$?; tail -4 $O/sparse.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o run -- python3 bench.py --steps 20 --warmup 3 \
    --no-cpu-baseline > $O/prof_c2.log 2>&1
rc=$?
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('C2', d['ms_per_step'], d['value'], r.get('frac'), r.get('kernel_avg_ms'))" $O/bench_c2.json
[ $rc -eq 0 ] || exit $rc
AB_OUT=r04s11/ab3 bash scripts/r04/ab.sh "--config c3 --steps 10 --warmup 2" \
    "--config c3 --steps 10 --warmup 2 --opt rare_flat=0" || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_variant.py -m gpu -x -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $O/variant.log 2>&1
rc=$?; tail -6 $O/variant.log; [ $rc -eq 0 ] || exit $rc
exit 0
