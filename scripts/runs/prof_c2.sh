set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c2 -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_c2.log 2>&1 || exit $?
find gpurun_out/prof_c2 -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/c2_kernel_stats.csv
