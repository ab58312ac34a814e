#!/bin/bash
# v5 sparse kernel on C2: E16 records vs word + set loads, chunk counts
set -o pipefail
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -k "kernel_v5" -x -q --timeout 300 --timeout-method thread > gpurun_out/v5_tests.log 2>&1 || { tail -30 gpurun_out/v5_tests.log; exit 1; }
tail -1 gpurun_out/v5_tests.log
export TMPDIR=/tmp
for cfg in "cp4 --opt sparse_kernel=5 --opt sparse_abl=3 --opt sparse_sun=4" "cp3 --opt sparse_kernel=5 --opt sparse_abl=3" "q2 --opt sparse_kernel=5 --opt sparse_abl=4 --opt sparse_sun=2" "q3 --opt sparse_kernel=5 --opt sparse_abl=4" "t2 --opt sparse_kernel=5 --opt sparse_abl=5 --opt sparse_sun=2" "t3 --opt sparse_kernel=5 --opt sparse_abl=5" "cp4b --opt sparse_kernel=5 --opt sparse_abl=3 --opt sparse_sun=4"; do
  set -- $cfg; n=$1; shift
  timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/v5c_$n -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/v5c_$n.json 2> gpurun_out/v5c_$n.err || { tail -3 gpurun_out/v5c_$n.err; exit 1; }
  python3 - "$n" <<'PY'
import csv, glob, sys, re, json
n = sys.argv[1]
d = json.load(open(f"gpurun_out/v5c_{n}.json"))
f = glob.glob(f"gpurun_out/v5c_{n}/**/*kernel_stats.csv", recursive=True)[0]
out = []
for r in csv.DictReader(open(f)):
    if "sparse_tile" in r['Name'] or "sparse_reduce" in r['Name']:
        out.append(f"{re.sub(r'gdist::[(]anonymous namespace[)]::', '', r['Name'])[5:25]} {float(r['AverageNs'])/1e6:.4f}")
print(f"{n:7s} step {d['ms_per_step']} ok {d['verified']['ok']} ", " | ".join(out))
PY
done
