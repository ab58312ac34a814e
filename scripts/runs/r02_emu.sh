#!/bin/bash
# Weak-scaling emulation on one GPU with the round-2 default path (v6, fused step): each rank's row block timed alone
set -o pipefail
export TMPDIR=/tmp
for g in 2 4 8; do
  EMU_G=$g EMU_KERNELS="" timeout -k 10 400 python3 -u scripts/emulate_ranks.py > gpurun_out/emu_G$g.log 2>&1 || { tail -5 gpurun_out/emu_G$g.log; exit 1; }
  tail -1 gpurun_out/emu_G$g.log
done
