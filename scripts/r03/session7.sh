#!/bin/bash
# Interleaved phased sketch kernel: its edge-case parity tests (window caps
# 1..600), an in-process A/B on C5 (default cap 300, caps 200 / 450, the V2
# whole-sketch kernel), then SQ/LDS counters of the default on 10,000 sketches.
# Outputs under gpurun_out/r03s7/.
set -o pipefail
O=gpurun_out/r03s7
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "sketch" --timeout 240 \
    --timeout-method thread -p no:cacheprovider > $O/t_sketch.log 2>&1 &&
AB_ROUNDS=2 AB_VARIANTS=default,sketch_cap=96,sketch_cap=160,sketch_cap=128+sketch_ring=512,sketch_phase=1 timeout -k 10 600 \
    python -u scripts/ab_sketch.py > $O/ab_c5.txt 2>&1 &&
AB_VARIANTS=default bash scripts/pmc_sketch.sh &&
python3 scripts/pmc_summary.py gpurun_out/pmc_sk1 gpurun_out/pmc_sk2 --kernel sketch_ > $O/pmc_phase.txt
rc=$?
tail -3 $O/t_sketch.log; cat $O/ab_c5.txt $O/pmc_phase.txt
exit $rc
