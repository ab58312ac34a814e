#!/bin/bash
# Round 6 session 18: the sketch ring kernel without static LDS (the ring at
# LDS address 0) and its 256-slot walk addressed by one v_perm_b32 a side
# (option sketch_perm) — sketch parity, in-process A/B on C5, the C5 line.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06s18
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -v --timeout 500 \
    --timeout-method thread -k "sketch or c5" -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/tests.log | head -20; exit $rc; }
AB_VARIANTS="default,sketch_perm=0" AB_ROUNDS=3 timeout -k 10 500 python -u scripts/ab_sketch.py > $O/ab_c5.txt 2>&1 || { tail -20 $O/ab_c5.txt; exit 1; }
tail -4 $O/ab_c5.txt
timeout -k 10 400 python -u bench.py --config c5 --steps 3 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err || exit 1
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('c5', d['ms_per_step'], d['value'], r.get('kernel_avg_ms'), r.get('frac'))" $O/bench_c5.json
