#!/bin/bash
# round 5 session 2: sparse + rare parity (lists padded to even length, the
# direct rare walk, the pipelined walk), A/B of the walk, the overhead split,
# the C4 slice with the direct rare walk and with the LDS-chunk walk
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05s2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_realistic.py -m gpu -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider -k "sparse or realistic or group or rare_tier_thresholds" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
AB_OUT=r05s2/ab AB_ENVS=";sparse_pipe=1;sparse_pipe=1,sparse_sun=2;sparse_sun=2" bash scripts/r05/ab_sparse.sh || exit $?
DIAG_OUT=r05s2/diag DIAG_VARIANTS="base d7 d8 d9" bash scripts/r05/diag.sh || exit $?
timeout -k 10 500 python -u bench.py --config c4 --rows 0:1024 --force-exchange --steps 5 --warmup 1 --no-cpu-baseline \
    > $O/bench_c4_direct.json 2> $O/bench_c4_direct.err || exit $?
python3 -c "import json; d=json.load(open('$O/bench_c4_direct.json')); r=d['roofline']; print('direct', d['ms_per_step'], [(o['kernel'][:20], o['kernel_avg_ms']) for o in r.get('other', [])], r['kernel_avg_ms'])"
timeout -k 10 500 python -u bench.py --config c4 --rows 0:1024 --force-exchange --steps 5 --warmup 1 --no-cpu-baseline \
    --opt rare_direct=0 > $O/bench_c4_lds.json 2> $O/bench_c4_lds.err || exit $?
python3 -c "import json; d=json.load(open('$O/bench_c4_lds.json')); r=d['roofline']; print('lds', d['ms_per_step'], [(o['kernel'][:20], o['kernel_avg_ms']) for o in r.get('other', [])], r['kernel_avg_ms'])"
