#!/bin/bash
# C2 A/B over context options: one bench line per VARIANTS entry
# (NAME=VALUE, "default" for none). Outputs under gpurun_out/r03/ab_c2/.
set -o pipefail
O=gpurun_out/r03/ab_c2
mkdir -p $O
for v in ${VARIANTS:-default}; do
    a=""; [ "$v" = default ] || a="--opt $v"
    timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline $a > $O/b_$v.json 2> $O/b_$v.err || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], d['ms_per_step'], d['value'], r.get('kernel_avg_ms'), r.get('step_kernel_span_ms'), d['verified']['ok'])" $O/b_$v.json
done
