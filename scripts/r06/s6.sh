#!/bin/bash
# Round 6 session 6: the four-column epilogue (parity in every mode, then the
# C3 line), the C4 slice (MFMA tiles back at 202 VGPRs) and its realistic
# twin's slice, and a two-rank rehearsal of the bench's multi-rank path on
# one GPU (host transport).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06s6
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_parity.py::test_distance_epilogue_modes tests/test_gpu_fullsize.py::test_c3_full_size_auto_vs_oracle \
    tests/test_gpu_realistic.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
line() {   # name, bench args
    local name=$1; shift
    timeout -k 10 600 python -u bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo "line $name failed"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1].split('/')[-1], d['ms_per_step'], d['value'], r.get('kernel_avg_ms'), r.get('frac'), r.get('traffic'), (d.get('cpu_baseline') or {}).get('value'), (d.get('verified') or {}).get('ok'))" $O/$name.json
}
line bench_c3 --config c3 --steps 50 --warmup 5
line bench_c3_epi1 --config c3 --steps 50 --warmup 5 --no-cpu-baseline --opt epilogue_rows=1
line bench_c4_slice1024 --config c4 --rows 0:1024 --force-exchange --steps 10 --warmup 3 --opt split_build=8
line bench_c4r_slice1024 --config c4r --rows 0:1024 --force-exchange --steps 10 --warmup 3 --opt split_build=8
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29561 bench.py --gpus 2 --transport host --same-device --steps 10 --warmup 3 --no-cpu-baseline \
    > $O/bench_c2_2rank_host.json 2> $O/bench_c2_2rank_host.err || { echo "2-rank rehearsal failed"; exit 1; }
tail -1 $O/bench_c2_2rank_host.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('2-rank', d['n_gpus'], d['ms_per_step'], d['value'], (d.get('verified') or {}).get('ok'))"
