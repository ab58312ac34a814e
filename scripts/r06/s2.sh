#!/bin/bash
# Round 6 session 2: the changed tests (poisoned replays, the R = 8 c4 case,
# AUTO on a gathered collection, the cached-oracle sweeps, C3/C4 at size),
# then an in-process A/B of the pipelined sparse walk on C2.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06s2
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread --durations=30 -p no:cacheprovider \
    tests/test_gpu_variant.py tests/test_multirank_gpu.py "tests/test_gpu_parity.py::test_sparse_complement_words_exact" \
    tests/test_jni_shim.py tests/test_gpu_parity.py::test_append_extends_segment_index \
    tests/test_gpu_fullsize.py::test_c3_full_size_auto_vs_oracle tests/test_gpu_fullsize.py::test_c4_full_size_slices_vs_oracle \
    > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
AB_ROUNDS=5 AB_ENVS="GDIST_SPARSE_PIPE=0;GDIST_SPARSE_PIPE=1,GDIST_SPARSE_SUN=2;GDIST_SPARSE_PIPE=0,GDIST_SPARSE_SUN=2;GDIST_SPARSE_PIPE=1" \
    timeout -k 10 300 python -u scripts/ab_env.py > $O/ab_pipe.txt 2> $O/ab_pipe.err
rc2=$?
cat $O/ab_pipe.txt | tail -12
exit $((rc | rc2))
