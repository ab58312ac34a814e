#!/bin/bash
# Round 6 session 12: the raw MFMA tiles' stage DMA spread between the MFMAs
# (one barrier a stage) and waves 4-7 at priority 1 (option
# bitset_mfma_sched), parity then in-process A/B on C3 and the C4 slice; the
# sparse chunk reduce with its finalize operands requested before the
# partials (C2 line + rocprofv3 kernel stats).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06s12
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/tests.log | head -20; exit $rc; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- \
    python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_c2_prof.json 2> $O/bench_c2_prof.err || exit $?
find $O -name "*kernel_trace.csv" -delete
AB_ENVS=";bitset_mfma_sched=1;bitset_mfma_sched=2;bitset_mfma_sched=3" AB_ROUNDS=3 \
    timeout -k 10 500 python -u scripts/r06/ab_c3.py > $O/ab_c3.txt 2>&1 || { tail -20 $O/ab_c3.txt; exit 1; }
tail -5 $O/ab_c3.txt
AB_ENVS=";bitset_mfma_sched=1;bitset_mfma_sched=3;bitset_mfma_splits=2" AB_ROUNDS=3 \
    timeout -k 10 700 python -u scripts/r05/ab_c4.py > $O/ab_c4.txt 2>&1 || { tail -20 $O/ab_c4.txt; exit 1; }
tail -5 $O/ab_c4.txt
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('c2', d['ms_per_step'], d['value'], r.get('kernel_avg_ms'), r.get('frac'))" $O/bench_c2.json
