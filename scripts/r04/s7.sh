#!/bin/bash
# Round 4 session 7: the whole -m gpu suite (without the C4 full-size test),
# smoke, the C2 line, the C3 line (2-byte and 4-byte rare members).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04s7
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider \
    --durations=15 -k "not c4_full" > $O/gputest.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $O/bench_c2.json 2> $O/bench_c2.err &&
timeout -k 10 400 python -u bench.py --config c3 --steps 10 --warmup 2 > $O/bench_c3.json 2> $O/bench_c3.err &&
timeout -k 10 400 python -u bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline --opt rare_u16=0 \
    > $O/bench_c3_u32.json 2> $O/bench_c3_u32.err
rc=$?
tail -3 $O/gputest.log; cat $O/smoke.log
for f in $O/bench_c2.json $O/bench_c3.json $O/bench_c3_u32.json; do
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], d['ms_per_step'], d['value'], r.get('frac'), r.get('kernel'), r.get('kernel_avg_ms'), (r.get('other') or {}).get('kernel_avg_ms'), d['end_to_end']['seconds'])" $f
done
exit $rc
