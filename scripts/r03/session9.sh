#!/bin/bash
# Triangle-only sketch launch: the sketch parity tests and the C5 full-size
# test, the C5 line; then the multi-rank bench path rehearsed on one GPU
# (2 and 4 ranks sharing device 0, host-staged exchange over gloo) on C2;
# the C2 line with rocprofv3 kernel stats (chunk reduce with 8 loads in flight).
# Outputs under gpurun_out/r03s9/.
set -o pipefail
O=gpurun_out/r03s9
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q -k "sketch or c5" \
    --timeout 300 --timeout-method thread -p no:cacheprovider > $O/t_sketch.log 2>&1 &&
timeout -k 10 400 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err &&
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29511 bench.py --gpus 2 --same-device --transport host --steps 10 --warmup 2 --no-cpu-baseline \
    > $O/bench_c2_2ranks.json 2> $O/bench_c2_2ranks.err &&
timeout -k 10 500 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
    --master-port 29512 bench.py --gpus 4 --same-device --transport host --steps 10 --warmup 2 --no-cpu-baseline \
    > $O/bench_c2_4ranks.json 2> $O/bench_c2_4ranks.err &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $O/bench_c2.json 2> $O/bench_c2.err &&
TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- \
    python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/prof_c2.json 2> $O/prof_c2.err
rc=$?
tail -3 $O/t_sketch.log
cut -c1-300 $O/bench_c5.json $O/bench_c2_2ranks.json $O/bench_c2_4ranks.json $O/bench_c2.json
grep -h "sparse_reduce\|sparse_tile" $O/prof_c2/run_kernel_stats.csv | cut -c1-60,200-320
exit $rc
