#!/bin/bash
# One GPU call: the parity suite, smoke, then the C2 bench line and the C4
# per-rank slice line (each step under its own time limit, stopping at the
# first failure). Outputs under gpurun_out/r03/.
set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 240 python -u scripts/diag/rare_table.py 300 200000 > gpurun_out/r03/rare_table.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider \
    --durations=20 > gpurun_out/r03/gputest.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/r03/bench_c2.json 2> gpurun_out/r03/bench_c2.err &&
timeout -k 10 400 python -u bench.py --config c4 --rows 0:64 --force-exchange --steps 2 --warmup 1 \
    --opt trace=1 > gpurun_out/r03/bench_c4_slice.json 2> gpurun_out/r03/bench_c4_slice.err
rc=$?
tail -3 gpurun_out/r03/gputest.log
cat gpurun_out/r03/bench_c2.json gpurun_out/r03/bench_c4_slice.json 2>/dev/null | cut -c1-400
exit $rc
