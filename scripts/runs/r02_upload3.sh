#!/bin/bash
# Overlapped upload v3 (runtime pageable copies in 64 MiB pieces from a host thread): pack parity, then C2 setup
# with / without the overlap (twice each, alternating), then the default bench line
set -o pipefail
D=gpurun_out/upload3
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_library.py -m gpu -x -v \
    -k "pack or golden or library" --timeout 300 --timeout-method thread > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -2 $D/tests.log
A="python bench.py --steps 10 --warmup 2 --no-cpu-baseline"
timeout -k 10 300 $A --opt trace=1 > $D/ov1.json 2> $D/ov1.err || { tail -20 $D/ov1.err; exit 1; }
timeout -k 10 300 $A --opt pack_overlap=0 --opt trace=1 > $D/ov0.json 2> $D/ov0.err || { tail -20 $D/ov0.err; exit 1; }
timeout -k 10 300 $A > $D/ov1b.json 2> $D/ov1b.err || { tail -20 $D/ov1b.err; exit 1; }
timeout -k 10 300 $A --opt pack_overlap=0 > $D/ov0b.json 2> $D/ov0b.err || { tail -20 $D/ov0b.err; exit 1; }
grep "gdist: pack" $D/ov1.err | head -8
grep "gdist: pack" $D/ov0.err | head -4
python3 -c "
import json
for f in ('ov1','ov0','ov1b','ov0b'):
    d=json.load(open('$D/'+f+'.json')); print(f, d['setup_s'], d['end_to_end']['pairs_per_s'], d['ms_per_step'])"
