#!/bin/bash
# round 5 session 16: dense tiles issued first (parity; C2-realistic, C3 and
# the C4 slice A/B in one process each)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05s16
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_options.py -m gpu -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider -k "sparse_complement or option or mfma" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
AB_CONFIG=c2r AB_ROUNDS=5 AB_ENVS=";dense_first=1" timeout -k 10 400 python -u scripts/ab_env.py > $O/ab_c2r.txt 2> $O/ab_c2r.err || exit $?
cat $O/ab_c2r.txt
AB_ENVS=";dense_first=1" timeout -k 10 400 python -u scripts/r05/ab_c4.py > $O/ab_c4.txt 2> $O/ab_c4.err || exit $?
grep -E "built|^\[" $O/ab_c4.txt
for o in "" "--opt dense_first=1"; do
  timeout -k 10 300 python -u bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline $o > $O/c3.json 2> $O/c3.err || exit $?
  python3 -c "import json; d=json.load(open('$O/c3.json')); print('c3 $o', d['ms_per_step'])"
done
