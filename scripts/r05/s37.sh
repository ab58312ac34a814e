#!/bin/bash
# round 5 session 37: C3's short walk with 256 / 1024-thread workgroups
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05s37
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_variant.py tests/test_gpu_options.py -m gpu -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider -k "grouped or option" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for o in "" "--opt variant_short_threads=256" "--opt variant_short_threads=1024" "" "--opt variant_short_threads=256" "--opt variant_short_threads=1024"; do
  timeout -k 10 300 python -u bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline $o > $O/c3.json 2> $O/c3.err || exit $?
  python3 -c "
import json; d=json.load(open('$O/c3.json')); r=d['roofline']
print('c3 [$o]', d['ms_per_step'], r['kernel_avg_ms'], [o['kernel_avg_ms'] for o in r.get('other', [])], d['verified']['ok'])"
done
