#!/bin/bash
# Group part evaluated per pair (no N x N table), sketch V2 default: the
# realistic + sketch parity tests, the c2r bench line, the C5 bench line and
# its rocprofv3 kernel stats. Outputs under gpurun_out/r03/s3/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03/s3
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_realistic.py tests/test_gpu_parity.py -m gpu -x -q \
    -k "realistic or sketch" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config c2r --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_c2r.json 2> $O/bench_c2r.err &&
timeout -k 10 400 python -u bench.py --config c5 --steps 3 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o run -- \
    python3 bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_c5.json 2> $O/prof_c5.err
rc=$?
tail -2 $O/t.log
for f in $O/bench_c2r.json $O/bench_c5.json; do
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['ms_per_step'], d['value'], d['roofline'].get('frac'), d.get('cpu_baseline'))" $f
done
exit $rc
