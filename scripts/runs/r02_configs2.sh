#!/bin/bash
# Round-end refresh of the other configs lines with the reworked pack (C2-realistic, C3); warmup past the graph capture
set -o pipefail
D=gpurun_out/configs2
mkdir -p $D
for c in c2r c3; do
  timeout -k 10 400 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > $D/line_$c.json 2> $D/line_$c.err || { tail -20 $D/line_$c.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$D/line_$c.json')); print('$c', d['value'], d['ms_per_step'], d['setup_s'], d.get('end_to_end_pairs_per_s'))"
done
