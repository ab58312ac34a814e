#!/bin/bash
# Rare row walk (upper-triangle skip, 16-byte member loads): the parity and
# full-size tests, then the C3 bench line. Outputs under gpurun_out/r03/c3r/.
set -o pipefail
O=gpurun_out/r03/c3r
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q \
    --timeout 500 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1
rc=$?; tail -2 $O/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err || exit $?
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['ms_per_step'], d['value'], d['roofline'].get('frac'), d.get('verified'))" $O/bench_c3.json
