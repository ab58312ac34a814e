set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
A="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ps_trace -o run -- $A > gpurun_out/ps_trace.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/ps_fetch -o run -- $A > gpurun_out/ps_fetch.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/ps_write -o run -- $A > gpurun_out/ps_write.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD --kernel-trace --output-format csv -d gpurun_out/ps_sq -o run -- $A > gpurun_out/ps_sq.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TA_TA_BUSY_sum GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/ps_tcp -o run -- $A > gpurun_out/ps_tcp.log 2>&1 || exit 1
echo prof done
