#!/bin/bash
# Ring kernel variant under test: sketch parity tests (+ C5 full size) and the C5 line.
set -o pipefail
O=gpurun_out/r03s16
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q -k "sketch or c5" --timeout 400 \
    --timeout-method thread -p no:cacheprovider > $O/t_sketch.log 2>&1 &&
timeout -k 10 400 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err
rc=$?
tail -2 $O/t_sketch.log; cut -c1-250 $O/bench_c5.json
exit $rc
