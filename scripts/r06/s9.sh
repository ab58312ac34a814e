#!/bin/bash
# Round 6 session 9: second-level variant keys (default) — parity (variant
# tier modes, split build, realistic twins), then the C4-realistic slice at
# the default Dmin and at Dmin 5000, the C4 slice (no keyless kmers: the
# same words), and C3-realistic (the grouped tier with second-level keys).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06s9
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_variant.py tests/test_gpu_realistic.py tests/test_gpu_parity.py::test_distance_epilogue_modes \
    > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
line() {   # name, bench args
    local name=$1; shift
    timeout -k 10 600 python -u bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo "line $name failed"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; v=d['config'].get('variant_tier') or {}; q=d['config'].get('rare_tier') or {}; print(sys.argv[1].split('/')[-1], d['ms_per_step'], d['value'], r.get('kernel'), r.get('kernel_avg_ms'), [(o.get('kernel','')[:20], o.get('kernel_avg_ms')) for o in r.get('other') or []], v.get('entries'), v.get('products'), q.get('records'), d['config'].get('bitset_words_per_set'), (d.get('verified') or {}).get('ok'))" $O/$name.json
    grep -E "keyless" $O/$name.err | head -2
}
A="--config c4r --rows 0:1024 --force-exchange --steps 10 --warmup 3 --opt split_build=8 --no-cpu-baseline --opt trace=1"
line c4r_default $A
line c4r_d5000 $A --opt variant_dmin=5000
line c3r_default --config c3r --steps 50 --warmup 5 --no-cpu-baseline --opt trace=1
line c3r_key1 --config c3r --steps 50 --warmup 5 --no-cpu-baseline --opt variant_key2=0
line c4_default --config c4 --rows 0:1024 --force-exchange --steps 10 --warmup 3 --opt split_build=8 --no-cpu-baseline --opt trace=1
