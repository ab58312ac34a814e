#!/bin/bash
# Sketch merge A/B: the sketch parity tests, then C5 with the round-2 merge
# (sketch_v2=0) and the V2 merge. Outputs under gpurun_out/r03/sk/.
set -o pipefail
O=gpurun_out/r03/sk
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k sketch --timeout 200 \
    --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1
rc=$?; tail -3 $O/t.log; [ $rc -eq 0 ] || exit $rc
VARIANTS=${VARIANTS:-"sketch_v2=0 sketch_v2=1"}
for v in $VARIANTS; do
    timeout -k 10 400 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --opt $v \
        > $O/b_$v.json 2> $O/b_$v.err || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['ms_per_step'], d['value'], d.get('verified'), d['roofline'].get('frac'))" $O/b_$v.json
done
