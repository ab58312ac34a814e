set -o pipefail
mkdir -p gpurun_out
for u in 8 12 16; do
GDIST_SPARSE_UNROLL=$u timeout -k 10 300 python bench.py --config c2 --steps 30 --no-cpu-baseline > gpurun_out/un_$u.json 2> gpurun_out/un.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/un_$u.json')); print('$u', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['verified']['ok'])"
done
