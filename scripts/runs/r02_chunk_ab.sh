#!/bin/bash
# Pack chunk size A/B (option pack_chunk: 2^30 default, 2^29, 2^28) on C2 with the overlapped upload
set -o pipefail
D=gpurun_out/chunk_ab
mkdir -p $D
A="python bench.py --steps 10 --warmup 2 --no-cpu-baseline"
for r in 1 2; do
  for c in 1073741824 536870912 268435456; do
    timeout -k 10 300 $A --opt pack_chunk=$c > $D/c${c}_$r.json 2> $D/c${c}_$r.err || { tail -20 $D/c${c}_$r.err; exit 1; }
  done
done
timeout -k 10 300 $A --opt pack_chunk=268435456 --opt trace=1 > $D/trace28.json 2> $D/trace28.err || exit 1
python3 -c "
import json,glob
for f in sorted(glob.glob('$D/c*.json')):
    d=json.load(open(f)); print(f.split('/')[-1], d['setup_s'], d['end_to_end']['pairs_per_s'], d['ms_per_step'])"
