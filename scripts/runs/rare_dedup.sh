set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "rare_tier or auto or single_rank or reps or row" > gpurun_out/t_rare.log 2>&1 || { tail -30 gpurun_out/t_rare.log; exit 1; }
tail -2 gpurun_out/t_rare.log
for c in c2 c3; do
  GDIST_TRACE=1 timeout -k 10 300 python bench.py --config $c --steps 10 --no-cpu-baseline > gpurun_out/b_$c.json 2> gpurun_out/b_$c.err || exit 1
done
GDIST_RARE_DEDUP=0 timeout -k 10 300 python bench.py --config c3 --steps 10 --no-cpu-baseline > gpurun_out/b_c3_nodedup.json 2> gpurun_out/b_c3_nodedup.err
