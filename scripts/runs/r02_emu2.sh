#!/bin/bash
# G=2 emulation: rank 0's block (the guide sets' rows) with the sparse plan traced, 8 vs 2 guides
set -o pipefail
export TMPDIR=/tmp
EMU_G=2 EMU_KERNELS="" GDIST_TRACE=1 timeout -k 10 400 python3 -u scripts/emulate_ranks.py > gpurun_out/emu2_g8.log 2>&1 || { tail -5 gpurun_out/emu2_g8.log; exit 1; }
grep -a "dense words\|sparse plan\|sparse chunks\|split model\|per-rank" gpurun_out/emu2_g8.log
EMU_G=2 EMU_KERNELS="" GDIST_GUIDES=2 timeout -k 10 400 python3 -u scripts/emulate_ranks.py > gpurun_out/emu2_g2.log 2>&1 || { tail -5 gpurun_out/emu2_g2.log; exit 1; }
tail -1 gpurun_out/emu2_g2.log
EMU_G=2 EMU_KERNELS="" GDIST_SPARSE_FUSED=0 timeout -k 10 400 python3 -u scripts/emulate_ranks.py > gpurun_out/emu2_nf.log 2>&1 || { tail -5 gpurun_out/emu2_nf.log; exit 1; }
tail -1 gpurun_out/emu2_nf.log
