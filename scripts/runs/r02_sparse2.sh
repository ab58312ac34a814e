#!/bin/bash
# A/B of the sparse tile kernel v1 (global loads per product) vs v2 (LDS-staged) on C2, after the sparse parity tests
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "sparse" -x -q --timeout 300 --timeout-method thread > gpurun_out/s2_tests.log 2>&1 || { tail -30 gpurun_out/s2_tests.log; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -k c2 -x -q --timeout 280 --timeout-method thread >> gpurun_out/s2_tests.log 2>&1 || { tail -30 gpurun_out/s2_tests.log; exit 1; }
for v in 1 2 1 2; do
  timeout -k 10 200 python bench.py --steps 30 --no-cpu-baseline --opt sparse_kernel=$v > gpurun_out/s2_v$v.json 2> gpurun_out/s2_v$v.err || { tail -20 gpurun_out/s2_v$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/s2_v$v.json'));print('v$v', d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['verified']['ok'])"
done
