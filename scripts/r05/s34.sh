#!/bin/bash
# round 5 session 34: the grouped rare tier probes its keyless share (falls
# back to the two tiers when keyless kmers dominate; packs them only below
# 1/4): parity, C3 with and without guide keys
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05s34
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_variant.py tests/test_gpu_options.py -m gpu -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for o in "" "--opt rare_group=2 --opt guides=0" "--opt rare_group=1 --opt guides=0" ""; do
  timeout -k 10 300 python -u bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline $o > $O/c3.json 2> $O/c3.err || exit $?
  python3 -c "
import json; d=json.load(open('$O/c3.json')); r=d['roofline']; c=d['config']
print('c3 [$o]', d['ms_per_step'], r['kernel_avg_ms'], c.get('variant_tier'), c.get('rare_tier'), d['verified']['ok'])"
done
