#!/bin/bash
# A/B: sparse tile kernel v1 vs v3 (16-byte records) at 4 / 6 products in flight, C2, after the sparse parity tests
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "sparse" -x -q --timeout 300 --timeout-method thread > gpurun_out/s3_tests.log 2>&1 || { tail -30 gpurun_out/s3_tests.log; exit 1; }
for rep in 1 2; do
for cfg in "1 6" "3 4" "3 6" "1 4"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --steps 30 --no-cpu-baseline --opt sparse_kernel=$1 --opt sparse_sun=$2 > gpurun_out/s3.json 2> gpurun_out/s3.err || { tail -20 gpurun_out/s3.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/s3.json'));print('v$1 sun$2', d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['verified']['ok'])"
done
done
