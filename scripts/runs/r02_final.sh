#!/bin/bash
# Round-2 measurement of the default path: smoke, the default bench line, rocprofv3 stats, FETCH/WRITE passes -> pmc json
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/final
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { tail -20 gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log
A="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final/trace -o run -- $A > gpurun_out/final/trace.json 2> gpurun_out/final/trace.log || exit 1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/final/fetch -o run -- $A > gpurun_out/final/fetch.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/final/write -o run -- $A > gpurun_out/final/write.log 2>&1 || exit 1
python3 scripts/pmc_json.py gpurun_out/final/fetch gpurun_out/final/write "sparse_tile_kernel<6, 8, false>" profiles/pmc_c2.json c2 1000
cp profiles/pmc_c2.json gpurun_out/final/pmc_c2.json
timeout -k 10 500 python bench.py > gpurun_out/final/bench_default.json 2> gpurun_out/final/bench_default.err || { tail -20 gpurun_out/final/bench_default.err; exit 1; }
cat gpurun_out/final/bench_default.json
