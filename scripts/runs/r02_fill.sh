#!/bin/bash
# bitset fill A/B: parity for the fill modes, then C2 setup with the merged-position fill (0) and the one-pass atomics (2)
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -k "fill or complement_words or prune or large_segments or full_size or fullsize or pack or rectangles or protein or empty or ambig or strand" > gpurun_out/fill_tests.log 2>&1 || { tail -30 gpurun_out/fill_tests.log; exit 1; }
tail -2 gpurun_out/fill_tests.log
for m in 0 2; do
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --opt fill_sort=$m --opt trace=1 > gpurun_out/fill_$m.json 2> gpurun_out/fill_$m.err || { tail -5 gpurun_out/fill_$m.err; exit 1; }
  grep -a "fill" gpurun_out/fill_$m.err | head -8
  python3 -c "import json,sys; d=json.load(open('gpurun_out/fill_$m.json')); print('$m', d.get('setup_s'), d.get('end_to_end'), d['ms_per_step'], d.get('verified'))"
done
