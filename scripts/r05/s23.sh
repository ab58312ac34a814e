#!/bin/bash
# round 5 session 23: raw MFMA stages of 8 words (64 KiB ring: two tile
# workgroups a CU, or one beside a walk workgroup): parity, then C3 and the
# C4 slice A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05s23
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider -k "mfma" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for o in "" "--opt bitset_mfma_km=2" "--opt bitset_mfma_km=2 --opt bitset_mfma_ns=3" "--opt bitset_mfma_km=2 --opt dense_first=0"; do
  timeout -k 10 300 python -u bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline $o > $O/c3.json 2> $O/c3.err || exit $?
  python3 -c "
import json; d=json.load(open('$O/c3.json')); r=d['roofline']
print('c3 [$o]', d['ms_per_step'], r['kernel_avg_ms'], [o['kernel_avg_ms'] for o in r.get('other', [])], d['verified']['ok'])"
done
AB_ENVS=";bitset_mfma_km=2;bitset_mfma_km=2,bitset_mfma_ns=3" timeout -k 10 500 python -u scripts/r05/ab_c4.py > $O/ab_c4.txt 2> $O/ab_c4.err || exit $?
grep -E "built|^\[" $O/ab_c4.txt
