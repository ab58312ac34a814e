set -o pipefail
mkdir -p gpurun_out
for g in 8 4 2; do
EMU_G=$g EMU_KERNELS="" timeout -k 10 400 python -u scripts/emulate_ranks.py > gpurun_out/emu_G$g.log 2>&1 || { tail -5 gpurun_out/emu_G$g.log; exit 1; }
tail -3 gpurun_out/emu_G$g.log
done
