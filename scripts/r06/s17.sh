#!/bin/bash
# Round 6 session 17: the e8m0 block scales of the FP4 MFMA (probe), then the
# bit-plane operands of the raw MFMA tiles (option bitset_mfma_plane: 5 VALU
# a dword instead of 7, per-step scales) — parity and in-process A/B on C3
# and the C4 slice.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06s17
mkdir -p $O
hipcc -O3 --offload-arch=gfx950 -Wno-unused-value scripts/microbench/fp4_scale_probe.hip -o $O/fp4_scale_probe || exit 1
timeout -k 10 60 $O/fp4_scale_probe > $O/fp4_scale_probe.txt 2>&1 || exit $?
rm -f $O/fp4_scale_probe
cat $O/fp4_scale_probe.txt
grep -q "bit planes under per-step scales: mismatches 0 " $O/fp4_scale_probe.txt || { echo "planes not exact: stop"; exit 0; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "mfma" -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/tests.log | head -20; exit $rc; }
AB_ENVS=";bitset_mfma_plane=1" AB_ROUNDS=4 timeout -k 10 400 python -u scripts/r06/ab_c3.py > $O/ab_c3.txt 2>&1 || { tail -20 $O/ab_c3.txt; exit 1; }
tail -2 $O/ab_c3.txt
AB_ENVS=";bitset_mfma_plane=1" AB_ROUNDS=3 timeout -k 10 600 python -u scripts/r05/ab_c4.py > $O/ab_c4.txt 2>&1 || { tail -20 $O/ab_c4.txt; exit 1; }
tail -2 $O/ab_c4.txt
