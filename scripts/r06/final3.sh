#!/bin/bash
# Round 6 final evidence, part 3 (the final tree): FETCH / WRITE passes of the
# MFMA tiles' default instantiation (bit-plane operands, spread DMA) on C3,
# C3-realistic and the C4 slice (profiles/pmc_{c3,c3r,c4}_mfma.json).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06final3
mkdir -p $O
pmc() {   # name, counter, bench args
    local name=$1 ctr=$2; shift 2
    timeout -k 10 400 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $O/$name -o run -- \
        python3 bench.py "$@" --no-cpu-baseline > $O/$name.json 2> $O/$name.err || { echo "pass $name failed"; exit 1; }
}
pmc c3_fetch FETCH_SIZE --config c3 --steps 5 --warmup 2
pmc c3_write WRITE_SIZE --config c3 --steps 5 --warmup 2
python3 scripts/pmc_json.py $O/c3_fetch $O/c3_write bitset_mfma_kernel $O/pmc_c3_mfma.json c3 10000 2 > /dev/null || exit 1
pmc c3r_fetch FETCH_SIZE --config c3r --steps 5 --warmup 2
pmc c3r_write WRITE_SIZE --config c3r --steps 5 --warmup 2
python3 scripts/pmc_json.py $O/c3r_fetch $O/c3r_write bitset_mfma_kernel $O/pmc_c3r_mfma.json c3r 10000 2 > /dev/null || exit 1
pmc c4_fetch FETCH_SIZE --config c4 --rows 0:1024 --force-exchange --steps 3 --warmup 2 --opt split_build=8
pmc c4_write WRITE_SIZE --config c4 --rows 0:1024 --force-exchange --steps 3 --warmup 2 --opt split_build=8
python3 scripts/pmc_json.py $O/c4_fetch $O/c4_write bitset_mfma_kernel $O/pmc_c4_mfma.json c4 100000 2 > /dev/null || exit 1
find $O -name "*counter_collection.csv" -delete
find $O -name "*kernel_trace.csv" -delete
for f in $O/pmc_*.json; do python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['kernel'][:50], d['hbm_bytes_x1'], d['hbm_bytes_x2'])" $f; done
