#!/bin/bash
# Round 6 session 5: the bench lines of C3 (MFMA tiles back at 202 VGPRs),
# the realistic twins C3r and C2r, C5; fresh FETCH / WRITE passes of C2's
# sparse tile kernel and C3r's walk and MFMA tiles (per-launch HBM bytes,
# both readings, exact kernel names).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06s5
mkdir -p $O
line() {   # name, bench args
    local name=$1; shift
    timeout -k 10 400 python -u bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo "line $name failed"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1].split('/')[-1], d['ms_per_step'], d['value'], r.get('kernel_avg_ms'), r.get('frac'), r.get('traffic'), (d.get('cpu_baseline') or {}).get('value'), (d.get('verified') or {}).get('ok'))" $O/$name.json
}
line bench_c3 --config c3 --steps 50 --warmup 5
line bench_c3r --config c3r --steps 50 --warmup 5
line bench_c2r --config c2r --steps 20 --warmup 3
pmc() {   # name, counter, bench args
    local name=$1 ctr=$2; shift 2
    timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $O/$name -o run -- \
        python3 bench.py "$@" --no-cpu-baseline > $O/$name.json 2> $O/$name.err || { echo "pass $name failed"; exit 1; }
}
pmc c2_fetch FETCH_SIZE --steps 5 --warmup 1
pmc c2_write WRITE_SIZE --steps 5 --warmup 1
python3 scripts/pmc_json.py $O/c2_fetch $O/c2_write sparse_tile_kernel $O/pmc_c2.json c2 1000 1 > /dev/null || exit 1
pmc c3r_fetch FETCH_SIZE --config c3r --steps 5 --warmup 2
pmc c3r_write WRITE_SIZE --config c3r --steps 5 --warmup 2
python3 scripts/pmc_json.py $O/c3r_fetch $O/c3r_write variant_short_kernel $O/pmc_c3r_variant_short.json c3r 10000 1 > /dev/null &&
python3 scripts/pmc_json.py $O/c3r_fetch $O/c3r_write bitset_mfma_kernel $O/pmc_c3r_mfma.json c3r 10000 2 > /dev/null || exit 1
find $O -name "*counter_collection.csv" -delete
find $O -name "*kernel_trace.csv" -delete
line bench_c5 --config c5 --steps 3 --warmup 1
