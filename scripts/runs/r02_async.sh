#!/bin/bash
# graph replay + asynchronous device-output calls: parity tests touching device outputs, then the C2 bench line and its timeline
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_options.py tests/test_bench_verify.py -x -q --timeout 300 --timeout-method thread > gpurun_out/as_tests.log 2>&1; tail -3 gpurun_out/as_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/as -o run -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/as.json 2> gpurun_out/as.err || { tail -5 gpurun_out/as.err; exit 1; }
timeout -k 10 300 python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/as2.json 2> gpurun_out/as2.err || { tail -5 gpurun_out/as2.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/as2.json'));print(d['ms_per_step'], d['value'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'], d['verified'])"
