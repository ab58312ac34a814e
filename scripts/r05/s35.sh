#!/bin/bash
# round 5 session 35: the C4 slice's variant walk slices a row (8-byte members)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05s35
mkdir -p $O
AB_ENVS=";variant_split=1;variant_split=4;variant_split=3" timeout -k 10 600 python -u scripts/r05/ab_c4.py > $O/ab_c4.txt 2> $O/ab_c4.err || exit $?
grep -E "built|^\[" $O/ab_c4.txt
