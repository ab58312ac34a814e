#!/bin/bash
# Round 4 session 41: the default C2 line unprofiled and the C2-realistic
# line on the final tree.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04s41
mkdir -p $O
timeout -k 10 300 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err || exit $?
timeout -k 10 400 python -u bench.py --config c2r --steps 10 --warmup 2 > $O/bench_c2r.json 2> $O/bench_c2r.err || exit $?
for f in bench_c2 bench_c2r; do
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], d['ms_per_step'], d['value'], r.get('kernel_avg_ms'), r.get('frac'), (d.get('end_to_end') or {}).get('seconds'))" $O/$f.json
done
