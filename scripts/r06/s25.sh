#!/bin/bash
# Round 6 session 25: C2-realistic's step with the round-6 MFMA tiles beside
# the sparse tiles: dense tiles issued first (option dense_first 1) and two
# K splits (bitset_mfma_splits 2) against the defaults (in-process A/B, counts
# checked equal).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06s25
mkdir -p $O
AB_CONFIG=c2r AB_ENVS=";dense_first=1;bitset_mfma_splits=2;dense_first=1,bitset_mfma_splits=2" AB_ROUNDS=7 \
    timeout -k 10 500 python -u scripts/ab_env.py > $O/ab_c2r.txt 2>&1 || { tail -20 $O/ab_c2r.txt; exit 1; }
tail -5 $O/ab_c2r.txt
