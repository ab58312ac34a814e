#!/bin/bash
# per-kernel time (rocprofv3 --kernel-trace --stats) of the C2 step for sparse kernel variants / guide counts
set -o pipefail
export TMPDIR=/tmp
run() {  # name, bench options...
  n=$1; shift
  timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/st_$n -o run -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/st_$n.json 2> gpurun_out/st_$n.err || { tail -5 gpurun_out/st_$n.err; exit 1; }
  echo "== $n $(python3 -c "import json;d=json.load(open('gpurun_out/st_$n.json'));print(d['ms_per_step'], d['config']['complement_sparse'], d['setup_s'])")"
  python3 - "$n" <<'PY'
import csv, glob, sys
n = sys.argv[1]
f = glob.glob(f"gpurun_out/st_{n}/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
for r in rows[:8]:
    print(f"  {r['Name'][:70]:70s} calls={r['Calls']:>5s} avg_ms={float(r['AverageNs'])/1e6:.4f} total_ms={float(r['TotalDurationNs'])/1e6:.2f}")
PY
}
run v1 --opt sparse_kernel=1
run v3 --opt sparse_kernel=3 --opt sparse_sun=4
run v3g4 --opt sparse_kernel=3 --opt sparse_sun=4 --opt guides=4
run v1g4 --opt sparse_kernel=1 --opt guides=4
