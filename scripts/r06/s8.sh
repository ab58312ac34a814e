#!/bin/bash
# Round 6 session 8: C4-realistic slice vs the variant tier's Dmin (the
# clade-specific kmers, held by ~7.5 K of 100 K genomes, are below N / 10 =
# 10 K, so their single-substitution variants have no dense neighbour and
# are keyless) and the keyless routing.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06s8
mkdir -p $O
line() {   # name, bench args
    local name=$1; shift
    timeout -k 10 600 python -u bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo "line $name failed"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; v=d['config'].get('variant_tier') or {}; q=d['config'].get('rare_tier') or {}; print(sys.argv[1].split('/')[-1], d['ms_per_step'], d['value'], r.get('kernel'), r.get('kernel_avg_ms'), [(o.get('kernel','')[:20], o.get('kernel_avg_ms')) for o in r.get('other') or []], v.get('entries'), v.get('products'), q.get('records'), d['config'].get('bitset_words_per_set'), (d.get('verified') or {}).get('ok'))" $O/$name.json
    grep -E "keyless" $O/$name.err | head -2
}
A="--config c4r --rows 0:1024 --force-exchange --steps 10 --warmup 3 --opt split_build=8 --no-cpu-baseline --opt trace=1"
line c4r_d5000_words $A --opt variant_dmin=5000 --opt variant_keyless_rare=0
line c4r_d5000_rare $A --opt variant_dmin=5000 --opt variant_keyless_rare=1
line c4r_d3000_auto $A --opt variant_dmin=3000
