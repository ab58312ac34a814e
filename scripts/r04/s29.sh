#!/bin/bash
# Round 4 session 29 (round-end evidence, part 2): the default bench line
# (C2) under rocprofv3 --kernel-trace --stats, its PMC passes (SQ / TA,
# FETCH_SIZE, WRITE_SIZE), and the C3 / C4-slice / C5 lines.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04s29
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- \
    python3 bench.py > $O/bench_c2.json 2> $O/bench_c2.err || exit $?
A2="--steps 5 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD \
    SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv \
    -d $O/c2_sq -o run -- python3 bench.py $A2 > $O/c2_sq.json 2> $O/c2_sq.err &&
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_WAIT_ANY \
    SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD TA_TA_BUSY_sum --kernel-trace --output-format csv \
    -d $O/c2_lds -o run -- python3 bench.py $A2 > $O/c2_lds.json 2> $O/c2_lds.err &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/c2_fetch -o run -- \
    python3 bench.py $A2 > $O/c2_fetch.json 2> $O/c2_fetch.err &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/c2_write -o run -- \
    python3 bench.py $A2 > $O/c2_write.json 2> $O/c2_write.err || exit $?
timeout -k 10 300 python -u bench.py --config c3 --steps 10 --warmup 2 > $O/bench_c3.json 2> $O/bench_c3.err || exit $?
timeout -k 10 300 python -u bench.py --config c5 --steps 3 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err || exit $?
timeout -k 10 500 python -u bench.py --config c4 --rows 0:1024 --force-exchange --steps 5 --warmup 1 --no-cpu-baseline \
    > $O/bench_c4_slice1024.json 2> $O/bench_c4_slice1024.err || exit $?
for f in bench_c2 bench_c3 bench_c5 bench_c4_slice1024; do
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], d['ms_per_step'], d['value'], r.get('kernel_avg_ms'), r.get('frac'), (d.get('end_to_end') or {}).get('seconds'))" $O/$f.json
done
