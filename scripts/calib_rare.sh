#!/bin/bash
# Rare-tier kernel calibration on the GPU box (repo root): scripts/calib_rare.py
# per case under rocprofv3 kernel trace + stats; outputs in gpurun_out/cal/<name>.
#   CAL_RUNS="name:case:T:rows ..." (default below)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
RUNS=${CAL_RUNS:-"c2:c2:-1:0:1 c3:c3:-1:0:1 c4s:c4s:-1:0:1 g8:g8:-1:0:1 g8T32:g8:32:0:1 g8T32last:g8:32:0.6464:1 g8last:g8:-1:0.6464:1"}
mkdir -p gpurun_out/cal
for r in $RUNS; do
    IFS=: read -r name case T a b <<< "$r"
    CAL_CASE=$case CAL_T=$T CAL_ROWS="$a:$b" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
        -d gpurun_out/cal/$name -o run -- python3 scripts/calib_rare.py > gpurun_out/cal/$name.log 2>&1 || exit $?
    echo "$name done"
done
