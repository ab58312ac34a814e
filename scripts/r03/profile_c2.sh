#!/bin/bash
# rocprofv3 evidence for the C2 bench line (round 3): kernel trace + stats of
# the default bench command, then FETCH_SIZE and WRITE_SIZE in separate PMC
# passes (kernel trace only), then the per-launch HBM bytes of the sparse
# tile kernel (scripts/pmc_json.py). Outputs under gpurun_out/r03/prof_*.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03
ARGS="--steps 20 --warmup 3 --no-cpu-baseline"
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_trace -o run -- \
    python3 bench.py $ARGS > $OUT/prof_trace.json 2> $OUT/prof_trace.err &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/prof_fetch -o run -- \
    python3 bench.py $ARGS > $OUT/prof_fetch.json 2> $OUT/prof_fetch.err &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/prof_write -o run -- \
    python3 bench.py $ARGS > $OUT/prof_write.json 2> $OUT/prof_write.err &&
python3 scripts/pmc_json.py $OUT/prof_fetch $OUT/prof_write "sparse_tile_kernel<3>" $OUT/pmc_c2.json c2 1000 &&
echo profile done
