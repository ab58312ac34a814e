#!/bin/bash
# Sparse tiles with the XCD-mapped chunk order (option sparse_xcd): the
# complement-word parity tests (xcd modes included), then C2 lines with and
# without it (interleaved) and a rocprofv3 stats + FETCH/WRITE profile with it
# (the default's: profiles/r03/s11/prof_default).  The XCD order rounds the chunk
# count up to a multiple of 8.
# Outputs under gpurun_out/r03s11/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03s11b
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_options.py -m gpu -x -q \
    -k "complement or option" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/t_xcd.log 2>&1 &&
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/b_default_$r.json 2> $O/b_default_$r.err &&
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --opt sparse_xcd=1 > $O/b_xcd_$r.json 2> $O/b_xcd_$r.err || exit 1
done &&
true &&
bash scripts/r03/profile.sh c2 1000 sparse_tile_kernel $O/prof_xcd "--opt sparse_xcd=1"
rc=$?
tail -3 $O/t_xcd.log
for f in $O/b_*.json; do
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], d['ms_per_step'], r.get('kernel_avg_ms'), r.get('frac'))" $f
done
cat $O/prof_default/pmc_c2.json $O/prof_xcd/pmc_c2.json 2>/dev/null
grep -h "sparse_tile" $O/prof_default/prof_trace/run_kernel_stats.csv $O/prof_xcd/prof_trace/run_kernel_stats.csv | cut -c1-40,190-300
exit $rc
