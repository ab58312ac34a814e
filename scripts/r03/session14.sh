#!/bin/bash
# HBM traffic (FETCH_SIZE x 2 + WRITE_SIZE, separate PMC passes) of the C5
# ring kernel and the C3 dense tile kernel (scripts/r03/profile.sh), then the
# C5 and C3 lines reading them (roofline.traffic). Outputs under gpurun_out/r03s14/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03s14
mkdir -p $O
bash scripts/r03/profile.sh c5 50000 sketch_ring_kernel $O/prof_c5 &&
bash scripts/r03/profile.sh c3 10000 bitset_tile_kernel2 $O/prof_c3 &&
timeout -k 10 400 python -u bench.py --config c5 --steps 3 --warmup 1 --pmc-json $O/prof_c5/pmc_c5.json \
    > $O/bench_c5.json 2> $O/bench_c5.err &&
timeout -k 10 400 python -u bench.py --config c3 --steps 10 --warmup 2 --pmc-json $O/prof_c3/pmc_c3.json \
    > $O/bench_c3.json 2> $O/bench_c3.err
rc=$?
cat $O/prof_c5/pmc_c5.json $O/prof_c3/pmc_c3.json
for f in $O/bench_c5.json $O/bench_c3.json; do
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['ms_per_step'], d['value'], json.dumps(d['roofline'])[:400])" $f
done
exit $rc
