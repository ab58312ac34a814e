#!/bin/bash
# round 5 session 32: the distance epilogue by rows (no 64-bit division per
# element, only the upper columns) and 16-byte zeroing: parity, C3 A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05s32
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_options.py tests/test_gpu_variant.py -m gpu -x -q --timeout 600 \
    --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for o in "" "--opt epilogue_rows=0" "" "--opt epilogue_rows=0"; do
  timeout -k 10 300 python -u bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline $o > $O/c3.json 2> $O/c3.err || exit $?
  python3 -c "
import json; d=json.load(open('$O/c3.json')); r=d['roofline']
print('c3 [$o]', d['ms_per_step'], r['kernel_avg_ms'], r.get('step_kernel_span_ms'), d['verified']['ok'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- \
    python3 bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline > $O/prof_c3.json 2> $O/prof_c3.err || exit $?
find $O/prof_c3 -name "*kernel_trace.csv" -delete
grep -E "epilogue|zero_upper" $O/prof_c3/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-120
