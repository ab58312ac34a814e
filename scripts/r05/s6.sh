#!/bin/bash
# round 5 session 6: persistent launch with a dynamic tail: parity, then A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05s6
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider -k "sparse_complement or graph_replay" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
AB_OUT=r05s6/ab AB_ENVS=";sparse_persist=1;sparse_persist=1,sparse_persist_tail=0;sparse_persist=1,sparse_persist_tail=40;sparse_persist=1,sparse_persist_tail=100" bash scripts/r05/ab_sparse.sh || exit $?
