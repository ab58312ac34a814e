#!/bin/bash
# Round 6 session 26: C3's MFMA K splits beside the one-slice short walk
# (bitset_mfma_splits 2 / 3 against the default 1), in-process A/B (counts
# checked equal), C3 and C3-realistic.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06s26
mkdir -p $O
AB_ENVS=";bitset_mfma_splits=2;bitset_mfma_splits=3" AB_ROUNDS=6 timeout -k 10 400 python -u scripts/r06/ab_c3.py > $O/ab_c3.txt 2>&1 || { tail -20 $O/ab_c3.txt; exit 1; }
tail -3 $O/ab_c3.txt
AB_CONFIG=c3r AB_ENVS=";bitset_mfma_splits=2" AB_ROUNDS=5 timeout -k 10 400 python -u scripts/r06/ab_c3.py > $O/ab_c3r.txt 2>&1 || { tail -20 $O/ab_c3r.txt; exit 1; }
tail -2 $O/ab_c3r.txt
