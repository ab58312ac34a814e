#!/bin/bash
# round 5 session 33: keyless variant kmers a word each (never sharing a
# word's list with unrelated kmers): parity; C3 with and without locus keys
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05s33
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_variant.py tests/test_gpu_options.py -m gpu -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for o in "" "--opt variant_pack_keyless=0" "--opt rare_group=1 --opt locus_order=0" "--opt rare_group=1 --opt locus_order=0 --opt variant_pack_keyless=0" "--opt rare_group=0 --opt locus_order=0"; do
  timeout -k 10 300 python -u bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline $o > $O/c3.json 2> $O/c3.err || exit $?
  python3 -c "
import json; d=json.load(open('$O/c3.json')); r=d['roofline']; c=d['config']
print('c3 [$o]', d['ms_per_step'], r['kernel_avg_ms'], c.get('variant_tier'), d['verified']['ok'])"
done
