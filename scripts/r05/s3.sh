#!/bin/bash
# round 5 session 3: parity of the persistent sparse launch (and the padded
# lists), then the C2 kernel: committed tree (before padding) vs this tree, persistent on/off
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05s3
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider -k "sparse_complement or graph_replay" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in head base; do
    for o in "" "sparse_persist=1"; do
      [ "$v" = head ] && [ -n "$o" ] && continue
      DIAG_OPTS="$o" timeout -k 10 200 python -u scripts/r05/diag_run.py $v 20 >> $O/diag.txt 2>> $O/diag.err || exit $?
      tail -1 $O/diag.txt
    done
  done
done
