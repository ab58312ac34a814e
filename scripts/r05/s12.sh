#!/bin/bash
# round 5 session 12: the MFMA tile-count criterion (parity; C2-realistic
# with the AND+popcount dense tiles vs MFMA forced), then the C4 slice on
# counters on the final variant walk (16-bit counters)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05s12
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_variant.py tests/test_gpu_options.py -m gpu -x -q \
    --timeout 300 --timeout-method thread -p no:cacheprovider -k "mfma or variant or option or rare or dense" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
AB_CONFIG=c2r AB_ROUNDS=5 AB_ENVS=";bitset_mfma=1" timeout -k 10 400 python -u scripts/ab_env.py > $O/ab_c2r.txt 2> $O/ab_c2r.err || exit $?
cat $O/ab_c2r.txt
bash scripts/r05/pmc_c4.sh $O/pmc "--opt serial_step=1" || exit $?
