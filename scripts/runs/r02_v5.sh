#!/bin/bash
# sparse parity tests, then v1 vs v5 (SUN = 4 / 6 / 8) kernel times on C2
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_realistic.py -k "sparse or realistic or graph" -x -q --timeout 300 --timeout-method thread > gpurun_out/v5_tests.log 2>&1 || { tail -30 gpurun_out/v5_tests.log; exit 1; }
tail -1 gpurun_out/v5_tests.log
for cfg in "v1 --opt sparse_kernel=1" "v5s4 --opt sparse_kernel=5 --opt sparse_sun=4" "v5s6 --opt sparse_kernel=5" "v5s4c --opt sparse_kernel=5 --opt sparse_sun=4 --opt sparse_abl=1" "v5s6c --opt sparse_kernel=5 --opt sparse_abl=1" "v5s4b --opt sparse_kernel=5 --opt sparse_sun=4"; do
  set -- $cfg; n=$1; shift
  timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/v5_$n -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/v5_$n.json 2> gpurun_out/v5_$n.err || { tail -3 gpurun_out/v5_$n.err; exit 1; }
  python3 - "$n" <<'PY'
import csv, glob, sys, re, json
n = sys.argv[1]
d = json.load(open(f"gpurun_out/v5_{n}.json"))
f = glob.glob(f"gpurun_out/v5_{n}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "sparse_tile" in r['Name']:
        print(f"{n:6s} step {d['ms_per_step']} ok {d['verified']['ok']} {re.sub(r'gdist::[(]anonymous namespace[)]::', '', r['Name'])[:40]:40s} {float(r['AverageNs'])/1e6:.4f} ms")
PY
done
