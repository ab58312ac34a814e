#!/bin/bash
# Round 6 final evidence, part 4: FETCH / WRITE passes of C2-realistic's
# sparse tile kernel and the C4-realistic slice's MFMA tiles (exact
# instantiations), then those two lines again with the passes in place.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06final4
mkdir -p $O
pmc() {   # name, counter, bench args
    local name=$1 ctr=$2; shift 2
    timeout -k 10 400 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $O/$name -o run -- \
        python3 bench.py "$@" --no-cpu-baseline > $O/$name.json 2> $O/$name.err || { echo "pass $name failed"; exit 1; }
}
pmc c2r_fetch FETCH_SIZE --config c2r --steps 5 --warmup 2
pmc c2r_write WRITE_SIZE --config c2r --steps 5 --warmup 2
python3 scripts/pmc_json.py $O/c2r_fetch $O/c2r_write sparse_tile_kernel $O/pmc_c2r.json c2r 1000 1 > /dev/null || exit 1
pmc c4r_fetch FETCH_SIZE --config c4r --rows 0:1024 --force-exchange --steps 3 --warmup 2 --opt split_build=8
pmc c4r_write WRITE_SIZE --config c4r --rows 0:1024 --force-exchange --steps 3 --warmup 2 --opt split_build=8
python3 scripts/pmc_json.py $O/c4r_fetch $O/c4r_write bitset_mfma_kernel $O/pmc_c4r_mfma.json c4r 100000 2 > /dev/null || exit 1
find $O -name "*counter_collection.csv" -delete
find $O -name "*kernel_trace.csv" -delete
cp $O/pmc_c2r.json profiles/pmc_c2r.json && cp $O/pmc_c4r_mfma.json profiles/pmc_c4r_mfma.json || exit 1
line() {   # name, bench args
    local name=$1; shift
    timeout -k 10 600 python -u bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo "line $name failed"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1].split('/')[-1], d['ms_per_step'], d['value'], r.get('kernel_avg_ms'), r.get('frac'), r.get('traffic'), (d.get('cpu_baseline') or {}).get('value'), (d.get('verified') or {}).get('ok'))" $O/$name.json
}
line bench_c2r --config c2r --steps 20 --warmup 3
line bench_c4r_slice1024 --config c4r --rows 0:1024 --force-exchange --steps 10 --warmup 3 --opt split_build=8
