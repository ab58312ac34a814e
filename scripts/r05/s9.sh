#!/bin/bash
# round 5 session 9: parity of the 16-bit rare counters and the heavy-row
# guard; the C4 slice on counters with each family alone (serial_step)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05s9
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_options.py -m gpu -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider -k "rare or option" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline > $O/c3.json 2> $O/c3.err || exit $?
timeout -k 10 300 python -u bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline --opt serial_step=1 > $O/c3_serial.json 2> $O/c3_serial.err || exit $?
timeout -k 10 300 python -u bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline --opt rare_c16=0 > $O/c3_c32.json 2> $O/c3_c32.err || exit $?
python3 - <<'PY'
import json
for f in ('c3', 'c3_serial', 'c3_c32'):
    d = json.load(open(f'gpurun_out/r05s9/{f}.json')); r = d['roofline']
    print(f, d['ms_per_step'], r['kernel'][:20], r['kernel_avg_ms'], [(o['kernel'][:20], o['kernel_avg_ms']) for o in r.get('other', [])])
PY
bash scripts/r05/pmc_c4.sh $O/pmc "--opt serial_step=1" || exit $?
