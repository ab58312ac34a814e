#!/bin/bash
# Round 6 final evidence, part 1 (the final tree): the whole -m gpu suite,
# smoke(), the C2 line (the bench default) and the same command under
# rocprofv3 --kernel-trace --stats, and fresh SQ counter passes of C2's
# sparse tile kernel (profiles/pmc_c2_sq.json).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06final1
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=30 \
    -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/smoke.log 2>&1 || exit $?
tail -2 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- \
    python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_c2_prof.json 2> $O/bench_c2_prof.err || exit $?
A2="--steps 5 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD \
    SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv \
    -d $O/c2_sq -o run -- python3 bench.py $A2 > $O/c2_sq.json 2> $O/c2_sq.err || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_WAIT_ANY \
    SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD TA_TA_BUSY_sum --kernel-trace --output-format csv \
    -d $O/c2_lds -o run -- python3 bench.py $A2 > $O/c2_lds.json 2> $O/c2_lds.err || exit $?
python3 scripts/pmc_sq_json.py $O/pmc_c2_sq.json c2 1000 sparse_tile_kernel $O/c2_sq $O/c2_lds > /dev/null || exit $?
find $O -name "*counter_collection.csv" -delete
find $O -name "*kernel_trace.csv" -delete
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('c2', d['ms_per_step'], d['value'], r.get('kernel_avg_ms'), r.get('frac'), r.get('traffic'), (d.get('cpu_baseline') or {}).get('value'), (d.get('verified') or {}).get('ok'))" $O/bench_c2.json
