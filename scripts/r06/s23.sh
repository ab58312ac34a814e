#!/bin/bash
# Round 6 session 23: the C4 slice's walk slices a row (option variant_split:
# 2 / 8 against the default 4) with the round-6 MFMA tiles beside them, and
# dense-first off; in-process A/B (counts checked equal).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06s23
mkdir -p $O
AB_ENVS=";variant_split=2;variant_split=8;dense_first=0" AB_ROUNDS=3 timeout -k 10 700 python -u scripts/r05/ab_c4.py > $O/ab_c4.txt 2>&1 || { tail -20 $O/ab_c4.txt; exit 1; }
tail -4 $O/ab_c4.txt
AB_ENVS=";variant_split=1;variant_split=4;dense_first=0" AB_ROUNDS=3 timeout -k 10 400 python -u scripts/r06/ab_c3.py > $O/ab_c3.txt 2>&1 || { tail -20 $O/ab_c3.txt; exit 1; }
tail -4 $O/ab_c3.txt
