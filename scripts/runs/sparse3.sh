set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "sparse or rare_tier or row or reps" > gpurun_out/t_sparse.log 2>&1 || { tail -40 gpurun_out/t_sparse.log; exit 1; }
tail -2 gpurun_out/t_sparse.log
timeout -k 10 300 python bench.py --config c2 --steps 20 --no-cpu-baseline > gpurun_out/b_c2.json 2> gpurun_out/b_c2.err || { tail -20 gpurun_out/b_c2.err; exit 1; }
