#!/bin/bash
# Round 6 session 13: the MFMA tiles' spread DMA as the default — the whole
# -m gpu suite, the C3 / C3r / C4 / C4r lines, fresh FETCH / WRITE passes of
# C3's and the C4 slice's MFMA instantiation; and a bound on C3's short-walk
# flush (the walk without its atomics into I, timing only: variant_short=9).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06s13
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=15 \
    -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/tests.log | head -20; exit $rc; }
AB_ENVS=";variant_short=9" AB_ROUNDS=3 timeout -k 10 400 python -u scripts/r06/ab_c3.py > $O/ab_c3_flush.txt 2>&1 || { tail -20 $O/ab_c3_flush.txt; exit 1; }
tail -3 $O/ab_c3_flush.txt
line() {   # name, bench args
    local name=$1; shift
    timeout -k 10 600 python -u bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo "line $name failed"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1].split('/')[-1], d['ms_per_step'], d['value'], r.get('kernel'), r.get('kernel_avg_ms'), r.get('frac'), [(o.get('kernel','')[:30], o.get('kernel_avg_ms'), o.get('frac')) for o in r.get('other') or []], (d.get('verified') or {}).get('ok'))" $O/$name.json
}
line bench_c3 --config c3 --steps 50 --warmup 5
line bench_c3r --config c3r --steps 50 --warmup 5
line bench_c4_slice1024 --config c4 --rows 0:1024 --force-exchange --steps 10 --warmup 3 --opt split_build=8
line bench_c4r_slice1024 --config c4r --rows 0:1024 --force-exchange --steps 10 --warmup 3 --opt split_build=8
pmc() {   # name, counter, bench args
    local name=$1 ctr=$2; shift 2
    timeout -k 10 400 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $O/$name -o run -- \
        python3 bench.py "$@" --no-cpu-baseline > $O/$name.json 2> $O/$name.err || { echo "pass $name failed"; exit 1; }
}
pmc c3_fetch FETCH_SIZE --config c3 --steps 5 --warmup 2
pmc c3_write WRITE_SIZE --config c3 --steps 5 --warmup 2
python3 scripts/pmc_json.py $O/c3_fetch $O/c3_write bitset_mfma_kernel $O/pmc_c3_mfma.json c3 10000 2 > /dev/null || exit 1
pmc c4_fetch FETCH_SIZE --config c4 --rows 0:1024 --force-exchange --steps 3 --warmup 2 --opt split_build=8
pmc c4_write WRITE_SIZE --config c4 --rows 0:1024 --force-exchange --steps 3 --warmup 2 --opt split_build=8
python3 scripts/pmc_json.py $O/c4_fetch $O/c4_write bitset_mfma_kernel $O/pmc_c4_mfma.json c4 100000 2 > /dev/null || exit 1
find $O -name "*counter_collection.csv" -delete
find $O -name "*kernel_trace.csv" -delete
