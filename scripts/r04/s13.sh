#!/bin/bash
# Round 4 session 13: counters. C2: SQ instruction pass (VALU per 64
# products of the reworked sparse walk) + FETCH_SIZE / WRITE_SIZE passes
# (profiles/pmc_c2.json); C3: kernel stats + FETCH / WRITE passes of the rare
# walk (pmc_c3_rare.json); the FETCH_SIZE calibration microbenchmark.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04s13
mkdir -p $O
AB_OUT=r04s13/ab_sun bash scripts/r04/ab.sh "--steps 20 --warmup 3" "--steps 20 --warmup 3 --opt sparse_sun=4" \
    "--steps 20 --warmup 3 --opt sparse_sun=2" || exit $?
A2="--steps 5 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- \
    python3 bench.py $A2 > $O/prof_c2.json 2> $O/prof_c2.err || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD \
    SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv \
    -d $O/c2_sq -o run -- python3 bench.py $A2 > $O/c2_sq.json 2> $O/c2_sq.err &&
python3 scripts/pmc_summary.py $O/c2_sq --kernel sparse_tile_kernel > $O/c2_sq.txt &&
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_WAIT_ANY \
    SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD TA_TA_BUSY_sum --kernel-trace --output-format csv \
    -d $O/c2_lds -o run -- python3 bench.py $A2 > $O/c2_lds.json 2> $O/c2_lds.err &&
python3 scripts/pmc_summary.py $O/c2_lds --kernel sparse_tile_kernel >> $O/c2_sq.txt &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/c2_fetch -o run -- \
    python3 bench.py $A2 > $O/c2_fetch.json 2> $O/c2_fetch.err &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/c2_write -o run -- \
    python3 bench.py $A2 > $O/c2_write.json 2> $O/c2_write.err &&
python3 scripts/pmc_json.py $O/c2_fetch $O/c2_write sparse_tile_kernel $O/pmc_c2.json c2 1000 &&
A3="--config c3 --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- \
    python3 bench.py $A3 > $O/prof_c3.json 2> $O/prof_c3.err &&
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/c3_fetch -o run -- \
    python3 bench.py $A3 > $O/c3_fetch.json 2> $O/c3_fetch.err &&
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/c3_write -o run -- \
    python3 bench.py $A3 > $O/c3_write.json 2> $O/c3_write.err &&
python3 scripts/pmc_json.py $O/c3_fetch $O/c3_write rare_rows_kernel $O/pmc_c3_rare.json c3 10000 &&
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES \
    SQ_WAIT_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/c3_sq -o run -- \
    python3 bench.py $A3 > $O/c3_sq.json 2> $O/c3_sq.err &&
python3 scripts/pmc_summary.py $O/c3_sq --kernel rare_rows_kernel > $O/c3_sq.txt &&
python3 scripts/pmc_summary.py $O/c3_sq --kernel bitset_mfma_kernel >> $O/c3_sq.txt &&
timeout -k 10 60 scripts/microbench/fetch_calib > $O/calib.txt 2>&1 &&
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/calib_fetch -o run -- \
    scripts/microbench/fetch_calib > $O/calib_fetch.log 2>&1
rc=$?
cat $O/c2_sq.txt $O/c3_sq.txt; cat $O/calib.txt; cat $O/pmc_c2.json $O/pmc_c3_rare.json 2>/dev/null | head -60
exit $rc
