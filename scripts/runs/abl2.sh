set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./scripts/microbench/lds_atomic > gpurun_out/lds_atomic.txt 2>&1
for a in 0 4; do
GDIST_SPARSE_ABL=$a timeout -k 10 300 python bench.py --config c2 --steps 20 --no-cpu-baseline > gpurun_out/abl_$a.json 2> gpurun_out/abl.err
done
true
