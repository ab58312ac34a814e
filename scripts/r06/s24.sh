#!/bin/bash
# Round 6 session 24: slices a row of the walks, more rounds — C4 slice
# variant_split 8 / 16 against the default 4, C3 short walk variant_split 1
# against the default 2 (in-process A/B, counts checked equal).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06s24
mkdir -p $O
AB_ENVS=";variant_split=8;variant_split=16" AB_ROUNDS=5 timeout -k 10 800 python -u scripts/r05/ab_c4.py > $O/ab_c4.txt 2>&1 || { tail -20 $O/ab_c4.txt; exit 1; }
tail -3 $O/ab_c4.txt
AB_ENVS=";variant_split=1" AB_ROUNDS=7 timeout -k 10 400 python -u scripts/r06/ab_c3.py > $O/ab_c3.txt 2>&1 || { tail -20 $O/ab_c3.txt; exit 1; }
tail -2 $O/ab_c3.txt
AB_CONFIG=c3r AB_ENVS=";variant_split=1" AB_ROUNDS=5 timeout -k 10 400 python -u scripts/r06/ab_c3.py > $O/ab_c3r.txt 2>&1 || { tail -20 $O/ab_c3r.txt; exit 1; }
tail -2 $O/ab_c3r.txt
