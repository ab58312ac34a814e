#!/bin/bash
# Round 4 session 27: the pack's code-bits sort (pack_code_sort) parity and
# setup A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04s27
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_options.py -m gpu -x -v --timeout 120 \
    --timeout-method thread -p no:cacheprovider -k "pack or option or k32 or sketch_build" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
AB_OUT=r04s27/abs bash scripts/r04/ab_setup.sh "" "--opt pack_code_sort=0" || exit $?
timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 3 --warmup 1 --opt trace=1 > $O/c2_trace.json 2> $O/c2_trace.err
