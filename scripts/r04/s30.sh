#!/bin/bash
# Round 4 session 30: C2 A/B 2 x 2 (default) vs 2 x 4 micro-tiles; setup A/B
# of the pack's code-bits sort; a C2 stage trace.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04s30
mkdir -p $O
AB_OUT=r04s30/ab bash scripts/r04/ab.sh "--steps 20 --warmup 3" "--steps 20 --warmup 3 --opt sparse_mt=4" || exit $?
AB_OUT=r04s30/abs bash scripts/r04/ab_setup.sh "" "--opt pack_code_sort=0" || exit $?
timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 3 --warmup 1 --opt trace=1 > $O/c2_trace.json 2> $O/c2_trace.err
