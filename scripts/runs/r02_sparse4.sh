#!/bin/bash
# sparse parity tests, then C2 step A/B: guides 2 vs 4 (4 = default), kernel v1 vs v3
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -k "sparse" -x -q --timeout 300 --timeout-method thread > gpurun_out/s4_tests.log 2>&1 || { tail -30 gpurun_out/s4_tests.log; exit 1; }
tail -2 gpurun_out/s4_tests.log
for cfg in "g4 --opt guides=4" "g2 --opt guides=2" "g4v3 --opt sparse_kernel=3 --opt sparse_sun=4"; do
  set -- $cfg; n=$1; shift
  timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s4_$n -o run -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/s4_$n.json 2> gpurun_out/s4_$n.err || { tail -5 gpurun_out/s4_$n.err; exit 1; }
  echo "== $n $(python3 -c "import json;d=json.load(open('gpurun_out/s4_$n.json'));print(d['ms_per_step'], d['config']['complement_sparse'], d['setup_s'], d['verified']['ok'])")"
  python3 - "$n" <<'PY'
import csv, glob, sys, re
n = sys.argv[1]
f = glob.glob(f"gpurun_out/s4_{n}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if int(r['Calls']) >= 20 and "gdist" in r['Name']:
        print(f"  {re.sub(r'gdist::[(]anonymous namespace[)]::', '', r['Name'])[:70]:70s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e6:.4f} ms")
PY
done
