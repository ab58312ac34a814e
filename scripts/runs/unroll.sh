set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "sparse" > gpurun_out/t_sparse.log 2>&1 || { tail -40 gpurun_out/t_sparse.log; exit 1; }
tail -1 gpurun_out/t_sparse.log
for u in 8 6 4; do
GDIST_SPARSE_UNROLL=$u timeout -k 10 300 python bench.py --config c2 --steps 30 --no-cpu-baseline > gpurun_out/un_$u.json 2> gpurun_out/un.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/un_$u.json')); print('$u', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['verified']['ok'])"
done
