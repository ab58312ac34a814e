#!/bin/bash
# Round 4 session 24: C2 A/B of the LDS-staged sparse walk (sparse_lds) with
# 2 / 3 / 4 slots a lane against the global walk.
set -o pipefail
export TMPDIR=/tmp
AB_OUT=r04s24/ab bash scripts/r04/ab.sh "--steps 20 --warmup 3" "--steps 20 --warmup 3 --opt sparse_lds=1" \
    "--steps 20 --warmup 3 --opt sparse_lds=1 --opt sparse_sun=4" "--steps 20 --warmup 3 --opt sparse_lds=1 --opt sparse_sun=2" || exit $?
