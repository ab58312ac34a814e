#!/bin/bash
# Overlapped chunk upload (option pack_overlap) + pack chunk summaries: parity (pack modes incl. small chunks,
# sparse modes, golden, full-size C2), then C2 setup with / without the overlap, then the default bench line
set -o pipefail
D=gpurun_out/upload
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_library.py -m gpu -x -v \
    -k "pack or sparse_complement or golden or full_size or library" --timeout 900 --timeout-method thread > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -2 $D/tests.log
A="python bench.py --steps 10 --warmup 2 --no-cpu-baseline"
timeout -k 10 300 $A --opt trace=1 > $D/ov1.json 2> $D/ov1.err || { tail -20 $D/ov1.err; exit 1; }
timeout -k 10 300 $A --opt pack_overlap=0 > $D/ov0.json 2> $D/ov0.err || { tail -20 $D/ov0.err; exit 1; }
timeout -k 10 300 $A > $D/ov1b.json 2> $D/ov1b.err || { tail -20 $D/ov1b.err; exit 1; }
grep "gdist: pack" $D/ov1.err | head -20
python3 -c "
import json
for f in ('ov1','ov0','ov1b'):
    d=json.load(open('$D/'+f+'.json')); print(f, d['setup_s'], d['end_to_end']['pairs_per_s'], d['ms_per_step'])"
timeout -k 10 500 python bench.py > $D/bench_default.json 2> $D/bench_default.err || { tail -20 $D/bench_default.err; exit 1; }
cat $D/bench_default.json
