#!/bin/bash
# round 5 session 4: parity (padded lists without the pipelined walk, the
# persistent launch with static batches, the variant walk across chunks),
# C2 kernel A/B (committed tree vs this tree vs persistent), C4 slice
# (variant prefetch; MFMA tiles grouped 4 x 8 so an XCD shares column panels)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05s4
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_variant.py -m gpu -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider -k "sparse_complement or graph_replay or variant" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in head base; do
    for o in "" "sparse_persist=1"; do
      [ "$v" = head ] && [ -n "$o" ] && continue
      DIAG_OPTS="$o" timeout -k 10 200 python -u scripts/r05/diag_run.py $v 20 >> $O/diag.txt 2>> $O/diag.err || exit $?
      tail -1 $O/diag.txt
    done
  done
done
for o in "" "--opt bitset_mfma_group=4"; do
  timeout -k 10 500 python -u bench.py --config c4 --rows 0:1024 --force-exchange --steps 5 --warmup 1 --no-cpu-baseline \
      $o > $O/c4.json 2> $O/c4.err || exit $?
  python3 -c "import json; d=json.load(open('$O/c4.json')); r=d['roofline']; print('$o', d['ms_per_step'], r['kernel'][:20], r['kernel_avg_ms'], [(x['kernel'][:20], x['kernel_avg_ms']) for x in r.get('other', [])])"
done
