#!/bin/bash
# Profile the bench workload on the GPU box (run from the repo root via gpurun).
#   pass 1: rocprofv3 --kernel-trace --stats   (per-kernel durations)
#   pass 2: rocprofv3 --pmc FETCH_SIZE         (HBM read bytes of the bench; own pass)
#   pass 3: rocprofv3 --pmc FETCH_SIZE         (calibration: build/membench, 16 GiB per
#           launch read by the same 128-B-run nt LDS-DMA pattern)
#   pass 4: rocprofv3 --pmc SQ counters        (wave/VALU/LDS activity; own pass)
set -u
TAG=${1:-r01}
ARGS=${2:---steps 20 --warmup 3 --no-cpu-baseline --no-host-inclusive}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py $ARGS > $OUT/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_calib -o run --output-format csv -- ./build/membench calib > $OUT/pmc_calib.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU -d $OUT/pmc_sq -o run --output-format csv -- python3 bench.py $ARGS > $OUT/pmc_sq.log 2>&1 || exit $?
echo done
