#!/bin/bash
# Round 4 session 35: parity of the galloping fill start (fill_guess) and
# the setup A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04s35
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_options.py -m gpu -x -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider -k "fill or option or k32" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
AB_OUT=r04s35/abs bash scripts/r04/ab_setup.sh "" "--opt fill_guess=1" || exit $?
timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 3 --warmup 1 --opt trace=1 --opt fill_guess=1 > $O/c2_trace.json 2> $O/c2_trace.err
