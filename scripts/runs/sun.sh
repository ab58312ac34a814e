set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "sparse or bitset or rare" > gpurun_out/t_sun.log 2>&1 || { tail -40 gpurun_out/t_sun.log; exit 1; }
tail -1 gpurun_out/t_sun.log
for x in 6 8 4 6 8 4; do
  GDIST_SPARSE_SUN=$x timeout -k 10 200 python bench.py --steps 30 --no-cpu-baseline > gpurun_out/sun_$x.json 2> gpurun_out/sun_$x.err || { tail -20 gpurun_out/sun_$x.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/sun_$x.json')); print('sun=$x', d['ms_per_step'], d['value']/1e9, d['roofline']['kernel_avg_ms'], d['verified']['ok'])"
done
