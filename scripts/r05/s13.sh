#!/bin/bash
# round 5 session 13: C3 with the row-major rare walk in line after the MFMA
# tiles (plain row stores) against beside them (atomic flush)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05s13
mkdir -p $O
for r in 1 2; do
  for o in "" "--opt rare_overlap=0"; do
    n=$([ -z "$o" ] && echo side || echo inline)
    timeout -k 10 300 python -u bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline $o > $O/c3_${n}_$r.json 2> $O/c3_${n}_$r.err || exit $?
    python3 -c "import json; d=json.load(open('$O/c3_${n}_$r.json')); r=d['roofline']; print('$n', d['ms_per_step'], r['kernel'][:20], r['kernel_avg_ms'], [(o['kernel'][:20], o['kernel_avg_ms']) for o in r.get('other', [])])"
  done
done
