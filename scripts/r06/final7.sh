#!/bin/bash
# Round 6 final evidence, part 7 (the final tree: C3's short walk one slice a
# row, the C4 variant walk's slices back at ~16 workgroups a CU after the
# C4-realistic regression in final6): the whole -m gpu suite, smoke(), the
# C4 and C4-realistic slice lines.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06final7
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=20 \
    -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/tests.log | head -20; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/smoke.log 2>&1 || exit $?
tail -2 $O/smoke.log
line() {   # name, bench args
    local name=$1; shift
    timeout -k 10 600 python -u bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo "line $name failed"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1].split('/')[-1], d['ms_per_step'], d['value'], r.get('kernel_avg_ms'), r.get('frac'), r.get('traffic'), (d.get('cpu_baseline') or {}).get('value'), (d.get('verified') or {}).get('ok'))" $O/$name.json
}
line bench_c4_slice1024 --config c4 --rows 0:1024 --force-exchange --steps 10 --warmup 3 --opt split_build=8
line bench_c4r_slice1024 --config c4r --rows 0:1024 --force-exchange --steps 10 --warmup 3 --opt split_build=8
