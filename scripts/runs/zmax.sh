set -o pipefail
mkdir -p gpurun_out
for z in default 100000 60 200; do
  if [ $z = default ]; then unset GDIST_SPARSE_ZMAX; else export GDIST_SPARSE_ZMAX=$z; fi
  timeout -k 10 300 python bench.py --config c2 --steps 10 --no-cpu-baseline > gpurun_out/zmax_$z.json 2> gpurun_out/zmax_$z.err || exit 1
done
