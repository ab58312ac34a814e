#!/bin/bash
# kernel times of the C2 setup for fill modes given as args
set -o pipefail
export TMPDIR=/tmp
for m in "$@"; do
  timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fillprof_$m -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --opt fill_sort=$m > gpurun_out/fillprof_$m.json 2> gpurun_out/fillprof_$m.err || { tail -3 gpurun_out/fillprof_$m.err; exit 1; }
  python3 - "$m" <<'PY'
import csv, glob, sys
m = sys.argv[1]
f = glob.glob(f"gpurun_out/fillprof_{m}/**/*kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r['TotalDurationNs']))
for r in rows[:8]:
    print(m, r['Name'][:60], r['Calls'], round(float(r['TotalDurationNs'])/1e6, 1), 'ms')
PY
done
