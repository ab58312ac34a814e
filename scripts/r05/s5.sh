#!/bin/bash
# round 5 session 5: sparse parity (committed walk + the persistent launch
# at 4 workgroups a CU), C2 kernel A/B: committed tree vs this tree vs persistent
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05s5
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 \
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
AB_OUT=r05s5/ab AB_ENVS=";sparse_persist=1" bash scripts/r05/ab_sparse.sh || exit $?
