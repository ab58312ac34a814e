#!/bin/bash
# round 5 session 28: MFMA tiles in 4 waves of 128 x 128 pairs (fewer
# fragment expansions per MFMA): parity, C3 and C4-slice A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05s28
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_options.py -m gpu -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider -k "mfma or option" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for o in "" "--opt bitset_mfma_waves=4" "" "--opt bitset_mfma_waves=4"; do
  timeout -k 10 300 python -u bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline $o > $O/c3.json 2> $O/c3.err || exit $?
  python3 -c "
import json; d=json.load(open('$O/c3.json')); r=d['roofline']
print('c3 [$o]', d['ms_per_step'], r['kernel_avg_ms'], [o['kernel_avg_ms'] for o in r.get('other', [])], d['verified']['ok'])"
done
AB_ENVS=";bitset_mfma_waves=4" timeout -k 10 500 python -u scripts/r05/ab_c4.py > $O/ab_c4.txt 2> $O/ab_c4.err || exit $?
grep -E "built|^\[" $O/ab_c4.txt
