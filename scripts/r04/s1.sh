#!/bin/bash
# Round 4 session 1: the per-step rare slots (no per-pair state between
# steps): the sparse / replay / options parity tests, the C2 line and its
# rocprofv3 kernel stats. Outputs under gpurun_out/r04s1/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04s1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_options.py -m gpu -x -q \
    -k "sparse or graph_replay or rare or options or plan" --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $O/gputest.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $O/bench_c2.json 2> $O/bench_c2.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- \
    python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/prof_c2.json 2> $O/prof_c2.err
rc=$?
tail -3 $O/gputest.log
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms_per_step'], d['value'], d['roofline'].get('frac'), d['end_to_end'])" $O/bench_c2.json
exit $rc
