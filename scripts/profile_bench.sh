#!/bin/bash
# rocprofv3 evidence for bench.py, run on the GPU box from the repo root:
#   1. kernel trace + stats of the default bench command (per-kernel durations)
#   2. separate PMC passes (FETCH_SIZE, then WRITE_SIZE) with kernel trace only
# Summaries land in gpurun_out/prof_*; copy the ones to keep into profiles/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ARGS=${BENCH_ARGS:-"--steps 5 --warmup 1 --no-cpu-baseline"}
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_trace -o run -- \
    python3 bench.py $ARGS > $OUT/prof_trace.log 2>&1 || exit $?
timeout -k 10 900 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/prof_fetch -o run -- \
    python3 bench.py $ARGS > $OUT/prof_fetch.log 2>&1 || exit $?
timeout -k 10 900 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/prof_write -o run -- \
    python3 bench.py $ARGS > $OUT/prof_write.log 2>&1 || exit $?
echo profile done
