#!/bin/bash
# Round 6 session 3: the pipelined 2 x 2 sparse walk as its own kernel
# instantiation (MT 3) against round 5's walk: in-process A/B on C2 and
# C2-realistic (step spans), then the bench line of both (the sparse kernel
# alone, HIP events), and the sparse parity sweep.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06s3
mkdir -p $O
E="GDIST_SPARSE_PIPE=0;;GDIST_SPARSE_PIPE=0,GDIST_SPARSE_SUN=2;GDIST_SPARSE_SUN=3"
AB_ROUNDS=9 AB_ENVS="$E" timeout -k 10 300 python -u scripts/ab_env.py > $O/ab_c2.txt 2> $O/ab_c2.err || exit $?
cat $O/ab_c2.txt
AB_CONFIG=c2r AB_ROUNDS=7 AB_ENVS="$E" timeout -k 10 300 python -u scripts/ab_env.py > $O/ab_c2r.txt 2> $O/ab_c2r.err || exit $?
cat $O/ab_c2r.txt
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_c2_pipe$r.json 2> $O/bench_c2_pipe$r.err || exit $?
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --opt sparse_pipe=0 > $O/bench_c2_nopipe$r.json 2> $O/bench_c2_nopipe$r.err || exit $?
done
for f in $O/bench_c2_*.json; do python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1].split('/')[-1], d['ms_per_step'], d['value'], r.get('kernel_avg_ms'), r.get('frac'))" $f; done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    "tests/test_gpu_parity.py::test_sparse_complement_words_exact" tests/test_gpu_parity.py::test_graph_replay_of_repeated_steps \
    tests/test_gpu_realistic.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; exit $rc
