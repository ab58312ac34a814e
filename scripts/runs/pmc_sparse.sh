set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
A="python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD --kernel-trace --output-format csv -d gpurun_out/pmc_sp1 -o run -- $A > gpurun_out/pmc_sp1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_VMEM SQ_ACCUM_PREV_HIRES --kernel-trace --output-format csv -d gpurun_out/pmc_sp2 -o run -- $A > gpurun_out/pmc_sp2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc_sp3 -o run -- $A > gpurun_out/pmc_sp3.log 2>&1 || exit 1
