#!/bin/bash
# C4 slice (1,024 rows x 100,000 columns) on counters:
# kernel trace + stats, FETCH_SIZE, WRITE_SIZE and two SQ/TA passes, each its
# own bench run, counters only on the step's kernels (--kernel-include-regex);
# per-launch JSON for the variant walk, the rare walk and the MFMA tiles, the
# raw counter CSVs deleted (gpurun_out/ travels back only under 64 MiB).
# Usage: pmc_c4.sh OUTDIR [EXTRA BENCH ARGS]
set -o pipefail
export TMPDIR=/tmp
OUT=$1; EXTRA=${2:-}
ARGS="--config c4 --rows 0:1024 --force-exchange --steps 3 --warmup 1 --no-cpu-baseline $EXTRA"
RX="variant_rows|rare_rows|bitset_mfma"
mkdir -p $OUT
run() {   # name, then rocprofv3 options
    local name=$1; shift
    timeout -k 10 420 rocprofv3 "$@" --output-format csv -d $OUT/$name -o run -- \
        python3 bench.py $ARGS > $OUT/$name.json 2> $OUT/$name.err || { echo "pass $name failed"; return 1; }
    echo "pass $name done"
}
run trace --kernel-trace --stats &&
run fetch --pmc FETCH_SIZE --kernel-trace --kernel-include-regex "$RX" &&
run write --pmc WRITE_SIZE --kernel-trace --kernel-include-regex "$RX" &&
run sq1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS \
    SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE TA_TA_BUSY_sum --kernel-trace --kernel-include-regex "$RX" &&
run sq2 --pmc SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU \
    SQ_WAIT_ANY --kernel-trace --kernel-include-regex "$RX" || exit 1
for k in variant_rows_kernel rare_rows bitset_mfma_kernel; do
    python3 scripts/pmc_json.py $OUT/fetch $OUT/write $k $OUT/pmc_c4_${k%_}.json c4 100000 1 > /dev/null &&
    python3 scripts/pmc_sq_json.py $OUT/pmc_c4_${k%_}_sq.json c4 100000 $k $OUT/sq1 $OUT/sq2 > /dev/null ||
    echo "no counters for $k"
done
# keep the stats of the trace pass and the JSONs; drop the per-dispatch CSVs
find $OUT -name "*counter_collection.csv" -delete
find $OUT -name "*kernel_trace.csv" -delete
echo pmc_c4 done
