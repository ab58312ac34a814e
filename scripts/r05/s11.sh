#!/bin/bash
# round 5 session 11: the wave walk's 16-bit counters / row slices (parity,
# then the C4 slice A/B in one process), then the C4 slice on counters with
# each family alone
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05s11
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_variant.py tests/test_gpu_options.py -m gpu -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
AB_ENVS=";variant_c16=1;variant_split=1;variant_c16=1,variant_split=1;variant_split=4" timeout -k 10 500 \
    python -u scripts/r05/ab_c4.py > $O/ab_c4.txt 2> $O/ab_c4.err || exit $?
cat $O/ab_c4.txt
bash scripts/r05/pmc_c4.sh $O/pmc "--opt serial_step=1" || exit $?
