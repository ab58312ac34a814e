#!/bin/bash
# Round 6 session 10: Dmin = N / 20 by default (the variant tier's dense
# threshold): realistic twin parity, the C4 full-size test (its tiers at the
# new default), the C4 and C4-realistic slices.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06s10
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_realistic.py tests/test_gpu_fullsize.py::test_c4_full_size_slices_vs_oracle \
    tests/test_multirank_gpu.py::test_multirank_c4_eight_ranks > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
line() {   # name, bench args
    local name=$1; shift
    timeout -k 10 600 python -u bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo "line $name failed"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; v=d['config'].get('variant_tier') or {}; print(sys.argv[1].split('/')[-1], d['ms_per_step'], d['value'], r.get('kernel'), r.get('kernel_avg_ms'), r.get('frac'), [(o.get('kernel','')[:20], o.get('kernel_avg_ms')) for o in r.get('other') or []], v.get('entries'), d['config'].get('bitset_words_per_set'), (d.get('cpu_baseline') or {}).get('value'), (d.get('verified') or {}).get('ok'))" $O/$name.json
}
line bench_c4_slice1024 --config c4 --rows 0:1024 --force-exchange --steps 10 --warmup 3 --opt split_build=8
line bench_c4r_slice1024 --config c4r --rows 0:1024 --force-exchange --steps 10 --warmup 3 --opt split_build=8
