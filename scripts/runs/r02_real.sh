#!/bin/bash
# realistic-collection parity tests, the C2-realistic bench line, then the v4/v1 PMC passes
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_realistic.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/real_tests.log 2>&1 || { tail -30 gpurun_out/real_tests.log; exit 1; }
grep -E "realistic|passed|failed" gpurun_out/real_tests.log
timeout -k 10 300 python bench.py --config c2r --steps 20 --no-cpu-baseline --opt trace=1 > gpurun_out/b_c2r.json 2> gpurun_out/b_c2r.err || { tail -5 gpurun_out/b_c2r.err; exit 1; }
grep "sparse plan" gpurun_out/b_c2r.err | head -1
python3 -c "import json;d=json.load(open('gpurun_out/b_c2r.json'));print('c2r', d['value'], d['ms_per_step'], d['config']['complement_sparse'], d['config']['rare_tier'], d['verified'])"
./scripts/runs/r02_pmc_v4.sh
