#!/bin/bash
# Sorted join launches cut at 2^31 work-items: the sorted / sketch parity
# tests; then the sketch kernel's SQ / LDS counters (scripts/pmc_sketch.sh,
# 10,000 sketches). Outputs under gpurun_out/r03/.
set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "sorted or sketch or device" \
    --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/r03/t_s5.log 2>&1
rc=$?; tail -2 gpurun_out/r03/t_s5.log; [ $rc -eq 0 ] || exit $rc
bash scripts/pmc_sketch.sh &&
python3 scripts/pmc_summary.py gpurun_out/pmc_sk1 gpurun_out/pmc_sk2 --kernel sketch_tile_kernel > gpurun_out/r03/pmc_sketch_v2.txt
rc=$?; cat gpurun_out/r03/pmc_sketch_v2.txt; exit $rc
