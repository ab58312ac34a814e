#!/bin/bash
# rocprofv3 evidence for one bench line: kernel trace + stats of the bench
# command, then FETCH_SIZE and WRITE_SIZE in separate PMC passes (kernel
# trace only), then the per-launch HBM bytes of the dominant kernel
# (scripts/pmc_json.py). Usage: profile.sh CONFIG N KERNEL OUTDIR [EXTRA BENCH ARGS]
set -o pipefail
export TMPDIR=/tmp
CFG=$1; N=$2; KERN=$3; OUT=$4; EXTRA=${5:-}
ARGS="--config $CFG --steps 20 --warmup 3 --no-cpu-baseline $EXTRA"
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_trace -o run -- \
    python3 bench.py $ARGS > $OUT/prof_trace.json 2> $OUT/prof_trace.err &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/prof_fetch -o run -- \
    python3 bench.py $ARGS > $OUT/prof_fetch.json 2> $OUT/prof_fetch.err &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/prof_write -o run -- \
    python3 bench.py $ARGS > $OUT/prof_write.json 2> $OUT/prof_write.err &&
python3 scripts/pmc_json.py $OUT/prof_fetch $OUT/prof_write "$KERN" $OUT/pmc_$CFG.json $CFG $N &&
echo profile $CFG done
