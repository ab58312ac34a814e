#!/bin/bash
# round 5 session 24: the C4 slice's MFMA tiles in G x 2G blocks (the row
# tiles of a column panel on one XCD: the panel fetched once per L2)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05s24
mkdir -p $O
AB_ENVS=";bitset_mfma_group=2;bitset_mfma_group=4;bitset_mfma_group=8" timeout -k 10 500 python -u scripts/r05/ab_c4.py > $O/ab_c4.txt 2> $O/ab_c4.err || exit $?
grep -E "built|^\[" $O/ab_c4.txt
