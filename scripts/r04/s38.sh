#!/bin/bash
# Round 4 session 38 (the final tree): the whole -m gpu suite, smoke, the
# default C2 line under rocprofv3 --kernel-trace --stats and its PMC passes.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04s38
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
    -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
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
    python3 bench.py $A2 > $O/c2_write.json 2> $O/c2_write.err
rc=$?
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(d['ms_per_step'], d['value'], r.get('kernel_avg_ms'), r.get('frac'), d['end_to_end']['seconds'])" $O/bench_c2.json
exit $rc
