#!/bin/bash
# Round 4 session 32: the sparse tile kernel's VALU without the trailing
# rare-row workgroups (sparse_rare 0 runs the rare tier in its own kernel),
# so the walk's own VALU per 64 products is separated from the recount's.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04s32
mkdir -p $O
A2="--steps 5 --warmup 1 --no-cpu-baseline --opt sparse_rare=0"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD \
    SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv \
    -d $O/c2_sq_norare -o run -- python3 bench.py $A2 > $O/c2_sq_norare.json 2> $O/c2_sq_norare.err &&
python3 scripts/pmc_sq_json.py $O/pmc_c2_sq_norare.json c2 1000 sparse_tile_kernel $O/c2_sq_norare
