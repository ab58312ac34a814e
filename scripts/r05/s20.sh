#!/bin/bash
# round 5 session 20: the grouped rare tier (16-kmer variant words, packed
# entries, a thread an entry): parity, then C3 with it (default) and without
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05s20
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_variant.py tests/test_gpu_options.py -m gpu -x -v --timeout 300 \
    --timeout-method thread -p no:cacheprovider -k "grouped or option or variant_tier_exact" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for o in "" "--opt rare_group=0" "--opt variant_split=2" "--opt variant_split=4" "--opt variant_c16=0"; do
  timeout -k 10 300 python -u bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline $o > $O/c3.json 2> $O/c3.err || exit $?
  python3 -c "
import json; d=json.load(open('$O/c3.json')); c=d['config']
print('c3 [$o]', d['ms_per_step'], c.get('variant_tier'), c.get('rare_tier'), d.get('kernel_ms_alone') or d.get('roofline'), d['verified']['ok'])"
done
