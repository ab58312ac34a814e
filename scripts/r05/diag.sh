#!/bin/bash
# the sparse kernel's cost decomposition (scripts/r05/diag_build.py variants)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${DIAG_OUT:-r05diag3}
mkdir -p $O
for r in 1 2; do
  for v in ${DIAG_VARIANTS:-base d5 d6 d7}; do
    DIAG_OPTS="$DIAG_OPTS" timeout -k 10 200 python -u scripts/r05/diag_run.py $v 20 >> $O/diag.txt 2>> $O/diag.err || exit $?
    tail -1 $O/diag.txt
  done
done
