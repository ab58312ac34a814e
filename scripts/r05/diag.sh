#!/bin/bash
# the sparse kernel's cost decomposition (scripts/r05/diag_build.py variants)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05diag2
mkdir -p $O
for r in 1 2; do
  for v in base d4 d5; do
    for o in "" "sparse_rare=0"; do
      DIAG_OPTS="$o" timeout -k 10 200 python -u scripts/r05/diag_run.py $v 20 >> $O/diag.txt 2>> $O/diag.err || exit $?
      tail -1 $O/diag.txt
    done
  done
done
