#!/bin/bash
# round 5 session 1: the JNI-harness GPU tests (genome cache, concat, sketch download),
# then the sparse kernel's cost decomposition
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05s1
timeout -k 10 300 python -u -m pytest tests/test_jni_shim.py -m gpu -x -v --timeout 200 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/r05s1/jni.log 2>&1
rc=$?; tail -3 gpurun_out/r05s1/jni.log; [ $rc -eq 0 ] || exit $rc
bash scripts/r05/diag.sh
