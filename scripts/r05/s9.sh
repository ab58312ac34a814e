#!/bin/bash
# round 5 session 9: parity of the 16-bit rare counters, the heavy-row guard
# and the variant walk's depth; C3 default / serial; the C4 slice A/B of the
# variant walk in one process; then the C4 slice on counters (families alone)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05s9
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_options.py tests/test_gpu_variant.py -m gpu \
    -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "rare or option or variant or split" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline > $O/c3.json 2> $O/c3.err || exit $?
timeout -k 10 300 python -u bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline --opt serial_step=1 > $O/c3_serial.json 2> $O/c3_serial.err || exit $?
python3 - <<'PY'
import json
for f in ('c3', 'c3_serial'):
    d = json.load(open(f'gpurun_out/r05s9/{f}.json')); r = d['roofline']
    print(f, d['ms_per_step'], r['kernel'][:20], r['kernel_avg_ms'], [(o['kernel'][:20], o['kernel_avg_ms']) for o in r.get('other', [])])
PY
AB_ENVS=";variant_depth=2;variant_depth=4;variant_small=0;variant_walk=0" timeout -k 10 500 python -u scripts/r05/ab_c4.py \
    > $O/ab_c4.txt 2> $O/ab_c4.err || exit $?
cat $O/ab_c4.txt
bash scripts/r05/pmc_c4.sh $O/pmc "--opt serial_step=1" || exit $?
