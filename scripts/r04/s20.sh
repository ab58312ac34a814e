#!/bin/bash
# Round 4 session 20: MFMA stage rings (2-word stages, 3 / 4 deep) — parity,
# then C3 and C4-slice A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04s20
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread \
    -p no:cacheprovider -k "dense_tiles_mfma" > $O/mfma.log 2>&1
rc=$?; tail -4 $O/mfma.log; [ $rc -eq 0 ] || exit $rc
AB_OUT=r04s20/ab3 bash scripts/r04/ab.sh "--config c3 --steps 10 --warmup 2 $BASE" \
    "--config c3 --steps 10 --warmup 2 $BASE --opt bitset_mfma_km=2 --opt bitset_mfma_ns=4" \
    "--config c3 --steps 10 --warmup 2 $BASE --opt bitset_mfma_km=2 --opt bitset_mfma_ns=3" \
    "--config c3 --steps 10 --warmup 2 $BASE --opt bitset_mfma_splits=1" \
    "--config c3 --steps 10 --warmup 2 $BASE --opt rare_overlap=0" || exit $?
for v in "" "--opt bitset_mfma_km=2 --opt bitset_mfma_ns=4"; do
    timeout -k 10 300 python -u bench.py --config c4 --rows 0:1024 --force-exchange --steps 5 --warmup 1 --no-cpu-baseline $BASE $v \
        > $O/c4.json 2> $O/c4.err || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('C4', sys.argv[2], d['ms_per_step'], r['kernel'][:24], r['kernel_avg_ms'], [(o['kernel'][:24], o['kernel_avg_ms']) for o in r.get('other', [])])" $O/c4.json "$v"
done
