#!/bin/bash
# Round 4 session 42: C2 chunk counts on the final walk.
set -o pipefail
export TMPDIR=/tmp
AB_OUT=r04s42/ab bash scripts/r04/ab.sh "--steps 20 --warmup 3" "--steps 20 --warmup 3 --opt sparse_chunks=75" \
    "--steps 20 --warmup 3 --opt sparse_chunks=93" "--steps 20 --warmup 3 --opt sparse_wg_per_cu=8" || exit $?
