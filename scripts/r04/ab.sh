#!/bin/bash
# A/B of bench lines in one call: each argument is a quoted set of bench.py
# arguments; three interleaved rounds. Outputs under gpurun_out/$AB_OUT/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${AB_OUT:-r04ab}
mkdir -p $O
for r in 1 2 3; do
  k=0
  for a in "$@"; do
    k=$((k+1))
    timeout -k 10 300 python -u bench.py --no-cpu-baseline $a > $O/v${k}_r$r.json 2> $O/v${k}_r$r.err || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], d['ms_per_step'], r.get('kernel_avg_ms'), r.get('step_kernel_span_ms'))" $O/v${k}_r$r.json "$a"
  done
done
