#!/bin/bash
# Profile the bench workload on the GPU box (run from the repo root via gpurun).
#   pass 1: rocprofv3 --kernel-trace --stats  (per-kernel durations)
#   pass 2: rocprofv3 --pmc FETCH_SIZE        (HBM read bytes; separate pass)
#   pass 3: rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum (request counts)
# plus a calibration kernel with a known byte count in the same pass structure.
set -u
TAG=${1:-r01}
ARGS=${2:---steps 20 --warmup 3 --no-cpu-baseline --no-host-inclusive}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py $ARGS > $OUT/pmc_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d $OUT/pmc_req -o run --output-format csv -- python3 bench.py $ARGS > $OUT/pmc_req.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_calib -o run --output-format csv -- python3 tools/calib_read.py > $OUT/pmc_calib.log 2>&1 || exit $?
echo done
