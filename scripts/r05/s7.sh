#!/bin/bash
# round 5 session 7: the split build (emulated shares on one GPU, the
# multi-rank worker on 2 and 3 host-transport ranks), release_codes, the
# rare walks; then the C4 slice with the 8-share build timed (trace on)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05s7
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_variant.py tests/test_gpu_options.py tests/test_multirank_gpu.py \
    tests/test_gpu_parity.py -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
    -k "variant or option or multirank or rare_tier or split or release or mfma or sketch" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --config c4 --rows 0:1024 --force-exchange --steps 5 --warmup 1 --no-cpu-baseline \
    --opt split_build=8 --opt trace=1 > $O/bench_c4_split8.json 2> $O/bench_c4_split8.err || exit $?
python3 -c "import json; d=json.load(open('$O/bench_c4_split8.json')); print(d['ms_per_step'], d['setup_s'])"
timeout -k 10 600 python -u bench.py --config c4 --rows 0:1024 --force-exchange --steps 5 --warmup 1 --no-cpu-baseline \
    --opt variant_walk=0 --opt bitset_mfma_raw=0 > $O/bench_c4_walk0.json 2> $O/bench_c4_walk0.err || exit $?
timeout -k 10 300 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || exit $?
timeout -k 10 300 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --opt sketch_super=0 > $O/bench_c5_s0.json 2> $O/bench_c5_s0.err || exit $?
timeout -k 10 300 python -u bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err || exit $?
timeout -k 10 300 python -u bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline --opt bitset_mfma_raw=0 > $O/bench_c3_nib.json 2> $O/bench_c3_nib.err || exit $?
python3 -c "
import json
for f in ('split8', 'walk0', 'c3', 'c3_nib', 'c5', 'c5_s0'):
    d = json.load(open('$O/bench_c4_%s.json' % f)); r = d['roofline']
    print(f, d['ms_per_step'], r.get('kernel'), r.get('kernel_avg_ms'), [(o['kernel'][:24], o['kernel_avg_ms']) for o in r.get('other', [])])
"
