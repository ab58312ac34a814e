#!/bin/bash
# Upload from registered host ranges (pack_overlap 2) vs runtime pageable pieces (1): pack parity, C2 setup A/B/A/B
set -o pipefail
D=gpurun_out/upload4
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_library.py -m gpu -x -v \
    -k "pack or golden or library" --timeout 300 --timeout-method thread > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -2 $D/tests.log
A="python bench.py --steps 10 --warmup 2 --no-cpu-baseline"
timeout -k 10 300 $A --opt pack_overlap=2 --opt trace=1 > $D/ov2.json 2> $D/ov2.err || { tail -20 $D/ov2.err; exit 1; }
timeout -k 10 300 $A > $D/ov1.json 2> $D/ov1.err || { tail -20 $D/ov1.err; exit 1; }
timeout -k 10 300 $A --opt pack_overlap=2 > $D/ov2b.json 2> $D/ov2b.err || { tail -20 $D/ov2b.err; exit 1; }
timeout -k 10 300 $A > $D/ov1b.json 2> $D/ov1b.err || { tail -20 $D/ov1b.err; exit 1; }
grep "gdist: pack" $D/ov2.err | head -8
python3 -c "
import json
for f in ('ov2','ov1','ov2b','ov1b'):
    d=json.load(open('$D/'+f+'.json')); print(f, d['setup_s'], d['end_to_end']['pairs_per_s'], d['ms_per_step'])"
