#!/bin/bash
# v5 sparse kernel on C2: chunk count sweep (workgroup rounds over 256 CUs x 4 slots), then PMC of v5 and v1
set -o pipefail
export TMPDIR=/tmp
for cfg in "c62 --opt sparse_kernel=5" "c28 --opt sparse_kernel=5 --opt sparse_chunks=28" "c40 --opt sparse_kernel=5 --opt sparse_chunks=40" "c56 --opt sparse_kernel=5 --opt sparse_chunks=56" "c85 --opt sparse_kernel=5 --opt sparse_chunks=85" "c113 --opt sparse_kernel=5 --opt sparse_chunks=113" "c28s4 --opt sparse_kernel=5 --opt sparse_chunks=28 --opt sparse_sun=4" "c113s4 --opt sparse_kernel=5 --opt sparse_chunks=113 --opt sparse_sun=4"; do
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
for v in 5 1; do
  A="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --opt sparse_kernel=$v"
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD --kernel-trace --output-format csv -d gpurun_out/pm5_$v/a -o run -- $A > gpurun_out/pm5_$v.a.log 2>&1 || exit 1
  timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INST_LEVEL_VMEM --kernel-trace --output-format csv -d gpurun_out/pm5_$v/b -o run -- $A > gpurun_out/pm5_$v.b.log 2>&1 || exit 1
  timeout -s KILL 150 rocprofv3 --pmc TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pm5_$v/c -o run -- $A > gpurun_out/pm5_$v.c.log 2>&1 || exit 1
  python3 scripts/pmc_summary.py gpurun_out/pm5_$v --kernel sparse_tile > gpurun_out/pm5_$v.txt
done
paste gpurun_out/pm5_5.txt gpurun_out/pm5_1.txt | awk '{print $3, $5, $10}'
