#!/bin/bash
# kernel 6 (micro-tiles) parity, then C2 A/B: shapes, slots in flight, dense-word absorb; alternated
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_realistic.py -k "sparse or realistic or graph" -x -q --timeout 300 --timeout-method thread > gpurun_out/v6_tests.log 2>&1 || { tail -30 gpurun_out/v6_tests.log; exit 1; }
tail -1 gpurun_out/v6_tests.log
timeout -k 10 120 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --opt trace=1 --opt sparse_absorb=0 > /dev/null 2> gpurun_out/v6_trace.err; grep -a "dense words\|sparse chunks\|sparse plan" gpurun_out/v6_trace.err || true
for cfg in "$@"; do
  set -- $cfg; n=$1; shift
  timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/v6_$n -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/v6_$n.json 2> gpurun_out/v6_$n.err || { tail -3 gpurun_out/v6_$n.err; exit 1; }
  python3 - "$n" <<'PY'
import csv, glob, sys, re, json
n = sys.argv[1]
d = json.load(open(f"gpurun_out/v6_{n}.json"))
f = glob.glob(f"gpurun_out/v6_{n}/**/*kernel_stats.csv", recursive=True)[0]
out = []
for r in csv.DictReader(open(f)):
    if int(r['Calls']) >= 12 and int(r['Calls']) < 40:
        m = re.search(r'::(\w+)(<[^(]*>)?\(', r['Name'])
        out.append(f"{(m.group(1) + (m.group(2) or ''))[:34] if m else r['Name'][:30]} {float(r['AverageNs'])/1e3:.1f}")
print(f"{n:8s} step {d['ms_per_step']} ok {d['verified']['ok']} ", " | ".join(out))
PY
done
