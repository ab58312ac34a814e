set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "sparse or bitset or rare" > gpurun_out/t_occ.log 2>&1 || { tail -40 gpurun_out/t_occ.log; exit 1; }
tail -1 gpurun_out/t_occ.log
for x in 3 8 3 8; do
  GDIST_SPARSE_OCC=$x timeout -k 10 200 python bench.py --steps 30 --no-cpu-baseline > gpurun_out/occ_$x.json 2> gpurun_out/occ_$x.err || { tail -20 gpurun_out/occ_$x.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/occ_$x.json')); print('occ=$x', d['ms_per_step'], d['value']/1e9, d['roofline']['kernel_avg_ms'], d['verified']['ok'])"
done
