#!/bin/bash
# sparse v2 timing ablations (C2): full / no walk / no fetch after the first window; v1 for reference
set -o pipefail
export TMPDIR=/tmp
for cfg in "v1 --opt sparse_kernel=1" "v2 --opt sparse_kernel=2" "v2nowalk --opt sparse_kernel=2 --opt sparse_abl=1" "v2nofetch --opt sparse_kernel=2 --opt sparse_abl=2"; do
  set -- $cfg; n=$1; shift
  timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab_$n -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/ab_$n.json 2> gpurun_out/ab_$n.err
  python3 - "$n" <<'PY'
import csv, glob, sys, re
n = sys.argv[1]
f = glob.glob(f"gpurun_out/ab_{n}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "sparse_tile" in r['Name']:
        print(f"{n:10s} {re.sub(r'gdist::[(]anonymous namespace[)]::', '', r['Name'])[:40]:40s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e6:.4f} ms")
PY
done
