#!/bin/bash
# Round 6 session 14: a bound on the C4 variant walk's flush (its atomics of
# each (row, slice, column chunk) into I skipped, timing only: variant_c16=9).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06s14
mkdir -p $O
AB_ENVS=";variant_c16=9" AB_ROUNDS=3 timeout -k 10 600 python -u scripts/r05/ab_c4.py > $O/ab_c4_flush.txt 2>&1 || { tail -20 $O/ab_c4_flush.txt; exit 1; }
tail -3 $O/ab_c4_flush.txt
