#!/bin/bash
# Rehearsal of the multi-rank bench path after the pack rework: 2 ranks sharing the one GPU, host-staged
# exchange (the driver's N>1 runs use RCCL on distinct GPUs), C2 shape at reduced size
set -o pipefail
D=gpurun_out/mr_bench
mkdir -p $D
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 2 --same-device --transport host --genomes 300 --length 400000 --steps 5 --warmup 1 --no-cpu-baseline \
    > $D/b2.json 2> $D/b2.err || { tail -30 $D/b2.err; exit 1; }
cat $D/b2.json
