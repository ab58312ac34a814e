#!/bin/bash
# Round 4 session 36: parity of the bits-operand MFMA tiles
# (bitset_mfma_bits) and the C3 / C4-slice A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04s36
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_options.py -m gpu -x -q --timeout 200 \
    --timeout-method thread -p no:cacheprovider -k "dense_tiles_mfma or option" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
AB_OUT=r04s36/ab bash scripts/r04/ab.sh "--config c3 --steps 10 --warmup 2" \
    "--config c3 --steps 10 --warmup 2 --opt bitset_mfma_bits=1" || exit $?
timeout -k 10 500 python -u bench.py --config c4 --rows 0:1024 --force-exchange --steps 5 --warmup 1 --no-cpu-baseline \
    --opt bitset_mfma_bits=1 > $O/c4_bits.json 2> $O/c4_bits.err || exit $?
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('c4 bits', d['ms_per_step'], d['value'], r.get('kernel_avg_ms'), [(o['kernel'][:30], o.get('kernel_avg_ms')) for o in r.get('other', [])])" $O/c4_bits.json
