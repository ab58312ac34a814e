#!/bin/bash
# C3 rare-tier threshold sweep now that the row-major rare kernel runs beside
# the dense tiles (rare_rows 4.47 ms vs tiles 3.58 ms at the cost model's T).
# Outputs under gpurun_out/r03s15/.
set -o pipefail
O=gpurun_out/r03s15
mkdir -p $O
for T in default 16 22 28 45; do
  if [ $T = default ]; then OPT=""; else OPT="--opt rare_t=$T"; fi
  timeout -k 10 300 python -u bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline $OPT \
      > $O/b_c3_$T.json 2> $O/b_c3_$T.err || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['config']['rare_tier']; print(sys.argv[1], d['ms_per_step'], d['value'], d['config']['bitset_words_per_set'], json.dumps(r)[:200])" $O/b_c3_$T.json
done
