#!/bin/bash
# Round 4 session 16: the C4 per-rank slice bench line (rank 0's first 64
# rows (and 1,024 rows) x 100,000 columns, the exchange through RCCL on a one-rank
# communicator, METHOD_AUTO -> the variant tier); the FP4 MFMA probe.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04s16
mkdir -p $O
timeout -k 10 60 scripts/microbench/fp4_probe > $O/fp4_probe.txt 2>&1
rc=$?; cat $O/fp4_probe.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py --config c4 --rows 0:64 --force-exchange --steps 5 --warmup 1 \
    > $O/bench_c4_slice.json 2> $O/bench_c4_slice.err &&
timeout -k 10 500 python -u bench.py --config c4 --rows 0:1024 --force-exchange --steps 5 --warmup 1 --no-cpu-baseline \
    > $O/bench_c4_slice1024.json 2> $O/bench_c4_slice1024.err
rc=$?
for f in $O/bench_c4_slice.json $O/bench_c4_slice1024.json; do
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(json.dumps(d)[:2500])" $f
done
exit $rc
