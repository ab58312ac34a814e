#!/bin/bash
# Round 6 session 21: EXPERIMENT — the MFMA tiles' second wave of every SIMD
# (waves 4-7) started ~64 / 128 cycles late each stage (a stagger of the
# SIMD partners' VALU and MFMA bursts; option bitset_mfma_stagger): in-process
# A/B on C3 and the C4 slice (counts checked equal).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06s21
mkdir -p $O
AB_ENVS=";bitset_mfma_stagger=1;bitset_mfma_stagger=2" AB_ROUNDS=4 timeout -k 10 400 python -u scripts/r06/ab_c3.py > $O/ab_c3.txt 2>&1 || { tail -20 $O/ab_c3.txt; exit 1; }
tail -3 $O/ab_c3.txt
AB_ENVS=";bitset_mfma_stagger=1;bitset_mfma_stagger=2" AB_ROUNDS=3 timeout -k 10 600 python -u scripts/r05/ab_c4.py > $O/ab_c4.txt 2>&1 || { tail -20 $O/ab_c4.txt; exit 1; }
tail -3 $O/ab_c4.txt
