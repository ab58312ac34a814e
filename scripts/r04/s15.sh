#!/bin/bash
# Round 4 session 15: C4 at its size on one GPU (tests/c4_worker.py: the
# consuming code all-gather on a one-rank RCCL communicator, METHOD_AUTO's
# variant-tier build from the gathered codes, rank 0's and the last rank's
# slices through the variant tier and the sorted join, three rows vs the
# oracle), then the C4 per-rank slice bench line through the variant tier.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04s15
mkdir -p $O
rm -f gpurun_out/c4_worker.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -q --timeout 890 --timeout-method thread \
    -p no:cacheprovider -k c4_full > $O/c4test.log 2>&1
rc=$?
cp gpurun_out/c4_worker.log $O/ 2>/dev/null
tail -5 $O/c4test.log; cat $O/c4_worker.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 280 python -u bench.py --config c4 --rows 0:64 --force-exchange --steps 5 --warmup 1 \
    > $O/bench_c4_slice.json 2> $O/bench_c4_slice.err
rc=$?
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(json.dumps(d)[:3000])" $O/bench_c4_slice.json
exit $rc
