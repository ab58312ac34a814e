#!/bin/bash
# round 5 session 29: C2 step vs the sparse chunk count (tile kernel + the
# chunk reduce that reads every chunk's partials), C2 and C2-realistic
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05s29
mkdir -p $O
AB_ROUNDS=5 AB_ENVS=";sparse_wg_per_cu=3;sparse_wg_per_cu=2;sparse_chunks=16;sparse_chunks=40" timeout -k 10 400 python -u scripts/ab_env.py > $O/ab_c2.txt 2> $O/ab_c2.err || exit $?
cat $O/ab_c2.txt | tail -8
AB_CONFIG=c2r AB_ROUNDS=5 AB_ENVS=";sparse_wg_per_cu=3;sparse_wg_per_cu=2;sparse_wg_per_cu=6" timeout -k 10 400 python -u scripts/ab_env.py > $O/ab_c2r.txt 2> $O/ab_c2r.err || exit $?
cat $O/ab_c2r.txt | tail -6
