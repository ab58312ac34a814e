#!/bin/bash
# in-process A/B of sparse-walk options on C2 (scripts/ab_env.py: interleaved rounds, counts checked equal)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${AB_OUT:-r05ab}
mkdir -p $O
AB_ROUNDS=${AB_ROUNDS:-5} AB_ENVS="$AB_ENVS" timeout -k 10 400 python -u scripts/ab_env.py > $O/ab.txt 2> $O/ab.err || exit $?
cat $O/ab.txt
