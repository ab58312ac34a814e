#!/bin/bash
# Round 4 session 31: the final tree's sparse parity + smoke, and C3's
# FETCH_SIZE / WRITE_SIZE passes for the FP4 MFMA dense tiles.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04s31
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_options.py -m gpu -x -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider -k "sparse_complement_words_exact or option or dense_tiles_mfma" \
    > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
A3="--config c3 --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/c3_fetch -o run -- \
    python3 bench.py $A3 > $O/c3_fetch.json 2> $O/c3_fetch.err &&
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/c3_write -o run -- \
    python3 bench.py $A3 > $O/c3_write.json 2> $O/c3_write.err || exit $?
python3 scripts/pmc_json.py $O/c3_fetch $O/c3_write bitset_mfma_kernel $O/pmc_c3_mfma.json c3 10000 2
