#!/bin/bash
# Row-major rare kernel beside the dense tiles (atomic row flush): the rare
# tier / full-size tests, then C3 with it in line (rare_overlap=0) and beside.
# Outputs under gpurun_out/r03/c3s/.
set -o pipefail
O=gpurun_out/r03/c3s
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q \
    -k "rare or c3 or auto or protein or sparse_equals" --timeout 500 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1
rc=$?; tail -2 $O/t.log; [ $rc -eq 0 ] || exit $rc
for v in rare_overlap=0 default; do
    a=""; [ "$v" = default ] || a="--opt $v"
    timeout -k 10 400 python -u bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline $a > $O/b_$v.json 2> $O/b_$v.err || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['ms_per_step'], d['value'], d['verified']['ok'])" $O/b_$v.json
done
