#!/bin/bash
# Round 4 session 17: the dense tiles on the matrix cores (FP4 MFMA) —
# parity first (the new test, then every bitset test), then C3 (A/B against
# the AND+popcount tiles) and the C4 slices.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04s17
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread \
    -p no:cacheprovider -k "dense_tiles_mfma" > $O/mfma.log 2>&1
rc=$?; tail -6 $O/mfma.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u scripts/r04/mfma_diag.py > $O/mfma_diag.txt 2>&1
rc=$?; cat $O/mfma_diag.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_variant.py tests/test_gpu_fullsize.py -m gpu -x -q \
    --timeout 300 --timeout-method thread -p no:cacheprovider -k "not c4_full" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
AB_OUT=r04s17/ab3 bash scripts/r04/ab.sh "--config c3 --steps 10 --warmup 2" \
    "--config c3 --steps 10 --warmup 2 --opt bitset_mfma=0" || exit $?
timeout -k 10 500 python -u bench.py --config c4 --rows 0:1024 --force-exchange --steps 5 --warmup 1 --no-cpu-baseline \
    > $O/bench_c4_slice1024.json 2> $O/bench_c4_slice1024.err
rc=$?
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(d['ms_per_step'], d['value'], r['kernel'], r['kernel_avg_ms'], [(o['kernel'][:30], o['kernel_avg_ms']) for o in r.get('other', [])])" $O/bench_c4_slice1024.json
exit $rc
