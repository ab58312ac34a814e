#!/bin/bash
# Round 4 session 10: the ring kernel's prefetched top-up (option
# sketch_prefetch) — merge edge cases vs the oracle, then a C5 A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04s10
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread \
    -p no:cacheprovider -k "sketch_merge_edges" > $O/edges.log 2>&1
rc=$?
tail -5 $O/edges.log
[ $rc -eq 0 ] || exit $rc
AB_OUT=r04s10/ab bash scripts/r04/ab.sh "--config c5 --steps 3 --warmup 1" "--config c5 --steps 3 --warmup 1 --opt sketch_prefetch=1"
