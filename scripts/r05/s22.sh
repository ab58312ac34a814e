#!/bin/bash
# round 5 session 22: grouped rare tier — parity (layout), C3 line with the
# CPU baseline, its rocprof kernel stats, and the short walk on counters
# (FETCH / WRITE / SQ passes, each family alone: serial_step)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05s22
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_variant.py tests/test_gpu_options.py -m gpu -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider -k "grouped or option" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --config c3 --steps 50 --warmup 5 > $O/bench_c3.json 2> $O/bench_c3.err || exit $?
python3 -c "import json; d=json.load(open('$O/bench_c3.json')); print('c3', d['ms_per_step'], d['value'], d['roofline']['kernel'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'], d['cpu_baseline'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- \
    python3 bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline > $O/prof_c3.json 2> $O/prof_c3.err || exit $?
ARGS="--config c3 --steps 5 --warmup 1 --no-cpu-baseline --opt serial_step=1"
RX="variant_short|bitset_mfma"
run() {
    local name=$1; shift
    timeout -k 10 300 rocprofv3 "$@" --kernel-include-regex "$RX" --output-format csv -d $O/$name -o run -- \
        python3 bench.py $ARGS > $O/$name.json 2> $O/$name.err || { echo "pass $name failed"; return 1; }
    echo "pass $name done"
}
run fetch --pmc FETCH_SIZE --kernel-trace &&
run write --pmc WRITE_SIZE --kernel-trace &&
run sq1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS \
    SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE TA_TA_BUSY_sum --kernel-trace &&
run sq2 --pmc SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU \
    SQ_WAIT_ANY --kernel-trace || exit 1
for k in variant_short_kernel bitset_mfma_kernel; do
    python3 scripts/pmc_json.py $O/fetch $O/write $k $O/pmc_c3_${k}.json c3 10000 1 > /dev/null &&
    python3 scripts/pmc_sq_json.py $O/pmc_c3_${k}_sq.json c3 10000 $k $O/sq1 $O/sq2 || echo "no counters for $k"
done
find $O -name "*counter_collection.csv" -delete
find $O -name "*kernel_trace.csv" -delete
echo s22 done
