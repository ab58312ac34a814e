#!/bin/bash
# Round 4 session 9: C3's rare walk on a roofline (rocprofv3 kernel stats,
# FETCH_SIZE and WRITE_SIZE passes of the C3 bench; profiles/pmc_c3_rare.json)
# and the FETCH_SIZE calibration microbenchmark (counters list, FETCH_SIZE
# and TCC_EA0_RDREQ passes).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04s9
mkdir -p $O
rocprofv3 -L > $O/counters_list.txt 2>&1 || true
A="--config c3 --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- \
    python3 bench.py $A > $O/prof_c3.json 2> $O/prof_c3.err &&
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/prof_c3_fetch -o run -- \
    python3 bench.py $A > $O/prof_c3_fetch.json 2> $O/prof_c3_fetch.err &&
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/prof_c3_write -o run -- \
    python3 bench.py $A > $O/prof_c3_write.json 2> $O/prof_c3_write.err &&
python3 scripts/pmc_json.py $O/prof_c3_fetch $O/prof_c3_write rare_rows_kernel $O/pmc_c3_rare.json c3 10000 &&
timeout -k 10 60 scripts/microbench/fetch_calib > $O/calib.txt 2>&1 &&
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/calib_fetch -o run -- \
    scripts/microbench/fetch_calib > $O/calib_fetch.log 2>&1 &&
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum --kernel-trace --output-format csv -d $O/calib_rdreq -o run -- \
    scripts/microbench/fetch_calib > $O/calib_rdreq.log 2>&1
rc=$?
cat $O/calib.txt; cat $O/pmc_c3_rare.json
grep -i "TCC_EA0_RD\|TCC_EA_RD" $O/counters_list.txt | head -20
exit $rc
