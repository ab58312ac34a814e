#!/bin/bash
# Pack chunk summaries (option pack_summary): parity (pack modes, sparse modes, golden, full-size C2 A/B),
# then the C2 setup stages with and without, then the default bench line
set -o pipefail
D=gpurun_out/packsum
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_library.py -m gpu -x -v \
    -k "pack or sparse_complement or golden or full_size or library" --timeout 900 --timeout-method thread > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -2 $D/tests.log
A="python bench.py --steps 10 --warmup 2 --no-cpu-baseline --opt trace=1"
timeout -k 10 300 $A > $D/sum1.json 2> $D/sum1.err || { tail -20 $D/sum1.err; exit 1; }
timeout -k 10 300 $A --opt pack_summary=0 > $D/sum0.json 2> $D/sum0.err || { tail -20 $D/sum0.err; exit 1; }
grep "gdist:" $D/sum1.err | head -40
python3 -c "
import json
for f in ('sum1','sum0'):
    d=json.load(open('$D/'+f+'.json')); print(f, d['setup_s'], d['end_to_end']['pairs_per_s'], d['ms_per_step'])"
timeout -k 10 500 python bench.py > $D/bench_default.json 2> $D/bench_default.err || { tail -20 $D/bench_default.err; exit 1; }
cat $D/bench_default.json
