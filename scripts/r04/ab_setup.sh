#!/bin/bash
# A/B of the setup (pack + represent + first call) of bench lines: each
# argument is a quoted set of bench.py arguments; three interleaved rounds.
# Outputs under gpurun_out/$AB_OUT/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${AB_OUT:-r04abs}
mkdir -p $O
for r in 1 2 3; do
  k=0
  for a in "$@"; do
    k=$((k+1))
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 5 --warmup 1 $a > $O/v${k}_r$r.json 2> $O/v${k}_r$r.err || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['setup_s'], d['end_to_end']['seconds'])" $O/v${k}_r$r.json "$a"
  done
done
