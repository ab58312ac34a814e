#!/bin/bash
# Round 4 session 18: the k=32 all-ones case under each fill route
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04s18
mkdir -p $O
timeout -k 10 120 python -u scripts/r04/mfma_diag.py > $O/mfma_diag.txt 2>&1
rc=$?; cat $O/mfma_diag.txt; exit $rc
