#!/bin/bash
# rocprofv3 passes over tools/crypt_bench.py (run from the repo root via gpurun): kernel
# trace + stats, SQ instruction/cycle counters, FETCH_SIZE, WRITE_SIZE (one pass each).
set -u
OUT=${1:-gpurun_out/cprof}
mkdir -p $OUT
export TMPDIR=/tmp
R=$PWD
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$OUT/trace -o run --output-format csv -- python3 $R/tools/crypt_bench.py --reps 3 > $R/$OUT/trace.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_LDS -d $R/$OUT/sq -o run --output-format csv -- python3 $R/tools/crypt_bench.py --reps 3 > $R/$OUT/sq.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $R/$OUT/fetch -o run --output-format csv -- python3 $R/tools/crypt_bench.py --reps 3 > $R/$OUT/fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $R/$OUT/write -o run --output-format csv -- python3 $R/tools/crypt_bench.py --reps 3 > $R/$OUT/write.log 2>&1 || exit 1
