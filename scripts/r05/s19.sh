#!/bin/bash
# round 5 session 19: C3 with its non-dense kmers in the variant tier (the
# kmers of one substitution grouped in a word: one product per shared
# substitution instead of one increment per shared kmer) against the rare tier
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05s19
mkdir -p $O
i=0
for o in "" "--opt variant=1 --opt rare_t=2 --opt variant_dmin=35" "--opt variant=1 --opt rare_t=2" "--opt variant=1 --opt rare_t=4 --opt variant_dmin=35"; do
  i=$((i+1))
  timeout -k 10 300 python -u bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline $o > $O/c3_$i.json 2> $O/c3_$i.err || exit $?
  python3 -c "
import json; d=json.load(open('$O/c3_$i.json')); c=d['config']
print('c3 [$o]', d['ms_per_step'], {k: c.get(k) for k in ('rare', 'variant', 'dense_words', 'width_words', 'kernel_ms_alone', 'verified')})"
done
