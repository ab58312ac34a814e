#!/bin/bash
# Re-entry check on a fresh box + the phased sketch kernel: its edge-case
# parity test first, the whole -m gpu suite, smoke, the default C2 bench line
# (fresh process: end-to-end figure), then C5 phased vs whole-sketch (V2).
# Outputs under gpurun_out/r03s6/.
set -o pipefail
O=gpurun_out/r03s6
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "sketch" --timeout 240 \
    --timeout-method thread -p no:cacheprovider > $O/t_sketch.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider \
    --durations=25 > $O/gputest.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $O/bench_c2.json 2> $O/bench_c2.err &&
timeout -k 10 400 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err &&
timeout -k 10 400 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --opt sketch_phase=0 \
    > $O/bench_c5_v2.json 2> $O/bench_c5_v2.err
rc=$?
tail -3 $O/t_sketch.log $O/gputest.log
cat $O/bench_c2.json $O/bench_c5.json $O/bench_c5_v2.json 2>/dev/null | cut -c1-500
exit $rc
