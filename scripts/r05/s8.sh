#!/bin/bash
# round 5 session 8: parity of the allocator / serial-step / chunk changes,
# the C4 slice with each family alone (serial_step) for both variant walks,
# the 8-share build traced (allocations), then the C4 counter passes
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05s8
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_variant.py tests/test_gpu_options.py -m gpu -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for v in 1 s0; do
  timeout -k 10 600 python -u bench.py --config c4 --rows 0:1024 --force-exchange --steps 5 --warmup 1 --no-cpu-baseline \
      --opt split_build=8 --opt trace=1 --opt serial_step=1 --opt variant_walk=${v#s} $([ $v = s0 ] && echo --opt variant_small=0 --opt variant_walk=1) > $O/c4_serial_w$v.json 2> $O/c4_serial_w$v.err || exit $?
  python3 -c "import json; d=json.load(open('$O/c4_serial_w$v.json')); r=d['roofline']; print('walk$v', d['ms_per_step'], r['kernel'][:20], r['kernel_avg_ms'], [(o['kernel'][:20], o['kernel_avg_ms']) for o in r.get('other', [])], d['setup_s'])"
done
timeout -k 10 600 python -u bench.py --config c4 --rows 0:1024 --force-exchange --steps 5 --warmup 1 --no-cpu-baseline \
    > $O/c4_default.json 2> $O/c4_default.err || exit $?
python3 -c "import json; d=json.load(open('$O/c4_default.json')); r=d['roofline']; print('default', d['ms_per_step'], r['kernel'][:20], r['kernel_avg_ms'], [(o['kernel'][:20], o['kernel_avg_ms']) for o in r.get('other', [])])"
bash scripts/r05/pmc_c4.sh $O/pmc || exit $?
