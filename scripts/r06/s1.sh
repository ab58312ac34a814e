#!/bin/bash
# Round 6 session 1: the whole -m gpu suite with per-test durations (the
# suite's budget), the C2 line, and a fresh LDS/SQ counter pass of C2's
# sparse tile kernel.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06s1
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
    --durations=80 -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err || exit $?
A2="--steps 5 --warmup 1 --no-cpu-baseline"
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_WAIT_ANY \
    SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD TA_TA_BUSY_sum --kernel-trace --output-format csv \
    -d $O/c2_lds -o run -- python3 bench.py $A2 > $O/c2_lds.json 2> $O/c2_lds.err
rc=$?
find $O -name "*kernel_trace.csv" -size +5M -delete
exit $rc
