#!/bin/bash
# round 5 session 25: 47-kmer variant words with 8-byte packed members (C4):
# parity (variant tier, multirank), the C4 slice A/B (packed vs the 4 + 8-byte
# arrays, in process) and its bench line
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05s25
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_variant.py tests/test_multirank_gpu.py tests/test_gpu_options.py -m gpu -x -v \
    --timeout 600 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
AB_ENVS=";variant_short=0" timeout -k 10 500 python -u scripts/r05/ab_c4.py > $O/ab_c4.txt 2> $O/ab_c4.err || exit $?
grep -E "built|^\[" $O/ab_c4.txt
timeout -k 10 500 python -u bench.py --config c4 --rows 0:1024 --force-exchange --steps 5 --warmup 1 --opt split_build=8 \
    --opt trace=1 > $O/bench_c4_slice1024.json 2> $O/bench_c4_slice1024.err || exit $?
grep -E "gdist: (variant|bitsets|fill|postings|range|build)" $O/bench_c4_slice1024.err > $O/c4_build_trace.txt
python3 -c "
import json; d=json.load(open('$O/bench_c4_slice1024.json')); r=d['roofline']
print('c4', d['ms_per_step'], d['value'], r['kernel'], r['kernel_avg_ms'], r['frac'], [(o['kernel'][:20], o['kernel_avg_ms']) for o in r.get('other', [])], d['verified'], d['config']['variant_tier'])"
