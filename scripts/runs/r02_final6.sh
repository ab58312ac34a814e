#!/bin/bash
# Round-2 measurement of the default path (sparse kernel v6): smoke, rocprofv3 stats, FETCH/WRITE -> pmc json,
# SQ/TA passes of the v6 kernel (limiter), the default bench line
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/final6
mkdir -p $D
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
A="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline"
K="sparse_tile_kernel5<3, 8, 1, 2, false>"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- $A > $D/trace.json 2> $D/trace.log || exit 1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $D/fetch -o run -- $A > $D/fetch.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $D/write -o run -- $A > $D/write.log 2>&1 || exit 1
python3 scripts/pmc_json.py $D/fetch $D/write "$K" profiles/pmc_c2.json c2 1000 && cp profiles/pmc_c2.json $D/ || exit 1
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD --kernel-trace --output-format csv -d $D/pa -o run -- $A > $D/pa.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INST_LEVEL_VMEM --kernel-trace --output-format csv -d $D/pb -o run -- $A > $D/pb.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $D/pc -o run -- $A > $D/pc.log 2>&1 || exit 1
python3 scripts/pmc_summary.py $D/pa $D/pb $D/pc --kernel "$K" > $D/pmc_v6.txt
timeout -k 10 500 python bench.py > $D/bench_default.json 2> $D/bench_default.err || { tail -20 $D/bench_default.err; exit 1; }
cat $D/bench_default.json
