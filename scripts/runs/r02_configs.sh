#!/bin/bash
# Round-2 lines of every single-GPU config after the v6 / fused changes: the default bench (C2, CPU legs),
# C2-realistic, C3, C5 (C4 slice through --n)
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/cfgs
mkdir -p $D
timeout -k 10 500 python bench.py > $D/c2_default.json 2> $D/c2_default.err || { tail -5 $D/c2_default.err; exit 1; }
timeout -k 10 300 python bench.py --config c2r --steps 20 --warmup 3 --no-cpu-baseline > $D/c2r.json 2> $D/c2r.err || { tail -5 $D/c2r.err; exit 1; }
timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline > $D/c3.json 2> $D/c3.err || { tail -5 $D/c3.err; exit 1; }
timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $D/c5.json 2> $D/c5.err || { tail -5 $D/c5.err; exit 1; }
for f in c2_default c2r c3 c5; do python3 -c "import json,sys;d=json.load(open('$D/$f.json'));print('$f', d['ms_per_step'], d['value'], d['config'].get('method'), d['verified']['ok'])"; done
