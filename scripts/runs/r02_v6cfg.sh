#!/bin/bash
# C2 or another config (BENCH_ARGS, e.g. "--config c2r"): trace of the split model, then per-config kernel breakdowns
set -o pipefail
export TMPDIR=/tmp
: # (parity: r02_v6.sh)

timeout -k 10 120 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline $BENCH_ARGS --opt trace=1 > /dev/null 2> gpurun_out/v6_trace.err; grep -a "dense words\|sparse chunks\|sparse plan\|split model" gpurun_out/v6_trace.err || true
for cfg in "$@"; do
  set -- $cfg; n=$1; shift
  timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/v6_$n -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline $BENCH_ARGS "$@" > gpurun_out/v6_$n.json 2> gpurun_out/v6_$n.err || { tail -3 gpurun_out/v6_$n.err; exit 1; }
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
