#!/bin/bash
# Round 4 session 5: the whole -m gpu suite + smoke with the per-step rare
# recount and the 2-byte rare members; the C2 and C3 lines (C3 with its rare
# kernel timed alone); C3 rocprofv3 kernel stats + FETCH / WRITE passes of
# the rare walk (rare_u16 on and off); the FETCH_SIZE calibration
# microbenchmark (counters list, FETCH_SIZE and TCC_EA0_RDREQ passes).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04s5
mkdir -p $O
rocprofv3 -L > $O/counters_list.txt 2>&1 || true
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider \
    --durations=15 -k "not c4_full" > $O/gputest.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $O/bench_c2.json 2> $O/bench_c2.err &&
timeout -k 10 400 python -u bench.py --config c3 --steps 10 --warmup 2 > $O/bench_c3.json 2> $O/bench_c3.err &&
timeout -k 10 400 python -u bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline --opt rare_u16=0 \
    > $O/bench_c3_u32.json 2> $O/bench_c3_u32.err &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- \
    python3 bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline > $O/prof_c3.json 2> $O/prof_c3.err &&
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/prof_c3_fetch -o run -- \
    python3 bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_c3_fetch.json 2> $O/prof_c3_fetch.err &&
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/prof_c3_write -o run -- \
    python3 bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_c3_write.json 2> $O/prof_c3_write.err &&
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/prof_c3u32_fetch -o run -- \
    python3 bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --opt rare_u16=0 \
    > $O/prof_c3u32_fetch.json 2> $O/prof_c3u32_fetch.err &&
timeout -k 10 60 scripts/microbench/fetch_calib > $O/calib.txt 2>&1 &&
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/calib_fetch -o run -- \
    scripts/microbench/fetch_calib > $O/calib_fetch.log 2>&1 &&
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum --kernel-trace --output-format csv -d $O/calib_rdreq -o run -- \
    scripts/microbench/fetch_calib > $O/calib_rdreq.log 2>&1 &&
timeout -k 10 1150 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -q --timeout 1150 --timeout-method thread \
    -p no:cacheprovider -k c4_full > $O/c4test.log 2>&1
rc=$?
tail -3 $O/gputest.log; tail -3 $O/c4test.log; cat gpurun_out/c4_worker.log; cat $O/smoke.log $O/calib.txt
for f in $O/bench_c2.json $O/bench_c3.json $O/bench_c3_u32.json; do
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], d['ms_per_step'], d['value'], r.get('frac'), r.get('kernel'), r.get('kernel_avg_ms'), (r.get('other') or {}).get('kernel_avg_ms'))" $f
done
exit $rc
