#!/bin/bash
# round 5 final C: the C3 and C4-slice lines again, each kernel family's
# roofline from its launches timed alone (bench.py: serial_step in the
# family-timing loop)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05final2
mkdir -p $O
timeout -k 10 300 python -u bench.py --config c3 --steps 10 --warmup 2 > $O/bench_c3.json 2> $O/bench_c3.err || exit $?
timeout -k 10 500 python -u bench.py --config c4 --rows 0:1024 --force-exchange --steps 5 --warmup 1 --opt split_build=8 \
    --opt trace=1 > $O/bench_c4_slice1024.json 2> $O/bench_c4_slice1024.err || exit $?
grep -E "gdist: (variant|bitsets|fill|postings|range|build)" $O/bench_c4_slice1024.err > $O/c4_build_trace.txt
for f in bench_c3 bench_c4_slice1024; do
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1].split('/')[-1], d['ms_per_step'], d['value'], r.get('kernel')[:30], r.get('kernel_avg_ms'), r.get('frac'), [(o['kernel'][:20], o['kernel_avg_ms'], o['frac']) for o in r.get('other', [])])" $O/$f.json
done
