#!/bin/bash
# Round 4 session 12: C4 diagnosis at size; the ring prefetch edge cases and a
# C5 A/B; setup A/B (10-bit radix passes) and C2 / C3 stage traces.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04s12
mkdir -p $O
timeout -k 10 500 python -u scripts/r04/c4_diag.py > $O/c4_out.txt 2> $O/c4_err.txt
rc=$?; tail -5 $O/c4_out.txt; grep -v "^RCCL\|NCCL\|LDS row" $O/c4_err.txt | tail -30; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread \
    -p no:cacheprovider -k "sketch_merge_edges" > $O/edges.log 2>&1
rc=$?; tail -3 $O/edges.log; [ $rc -eq 0 ] || exit $rc
AB_OUT=r04s12/ab bash scripts/r04/ab.sh "--config c5 --steps 3 --warmup 1" \
    "--config c5 --steps 3 --warmup 1 --opt sketch_prefetch=1" || exit $?
AB_OUT=r04s12/abs bash scripts/r04/ab_setup.sh "" "--opt sort_radix=10" || exit $?
timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 3 --warmup 1 --opt trace=1 > $O/c2_trace.json 2> $O/c2_trace.err &&
timeout -k 10 200 python -u bench.py --config c3 --no-cpu-baseline --steps 3 --warmup 1 --opt trace=1 > $O/c3_trace.json 2> $O/c3_trace.err
