#!/bin/bash
# Round 6 session 11 (checkpoint): the whole -m gpu suite with durations,
# smoke(), the C2 line.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06s11
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=25 \
    -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/smoke.log 2>&1 || exit $?
tail -2 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err || exit $?
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(d['ms_per_step'], d['value'], r.get('kernel_avg_ms'), r.get('frac'), r.get('traffic'), r.get('traffic_readings'), (d.get('cpu_baseline') or {}).get('value'), d.get('verified'))" $O/bench_c2.json
