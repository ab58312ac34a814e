#!/bin/bash
# round 5 session 14: C2-realistic — MFMA K splits for its 10 tiles, then
# the sparse tile kernel's HBM traffic (FETCH / WRITE passes on the bench)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05s14
mkdir -p $O
AB_CONFIG=c2r AB_ROUNDS=5 AB_ENVS=";bitset_mfma_splits=30;bitset_mfma_splits=60;bitset_mfma_splits=8" \
    timeout -k 10 400 python -u scripts/ab_env.py > $O/ab_c2r.txt 2> $O/ab_c2r.err || exit $?
cat $O/ab_c2r.txt
ARGS="--config c2r --steps 10 --warmup 2 --no-cpu-baseline"
RX="sparse_tile|bitset_mfma|sparse_reduce"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --kernel-include-regex "$RX" --output-format csv -d $O/fetch -o run -- \
    python3 bench.py $ARGS > $O/fetch.json 2> $O/fetch.err || exit $?
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --kernel-include-regex "$RX" --output-format csv -d $O/write -o run -- \
    python3 bench.py $ARGS > $O/write.json 2> $O/write.err || exit $?
for k in sparse_tile_kernel bitset_mfma_kernel sparse_reduce_kernel; do
  python3 scripts/pmc_json.py $O/fetch $O/write $k $O/pmc_c2r_$k.json c2r 1000 1 || echo "no counters for $k"
done
find $O -name "*counter_collection.csv" -delete
find $O -name "*kernel_trace.csv" -delete
