set -o pipefail
mkdir -p gpurun_out
for a in 0 1 2 3; do
GDIST_SPARSE_ABL=$a timeout -k 10 300 python bench.py --config c2 --steps 20 --no-cpu-baseline > gpurun_out/abl_$a.json 2> gpurun_out/abl.err
done
true
