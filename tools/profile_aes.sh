#!/bin/bash
# rocprofv3 over tools/crypt_bench.py --algo AES256-GCM-HMAC-SHA256 (run from the repo root via
# gpurun): kernel trace + stats, then one SQ counter pass (VALU / LDS instructions, LDS bank
# conflict cycles against all LDS-array cycles).
set -u
OUT=${1:-gpurun_out/aprof}
mkdir -p $OUT
export TMPDIR=/tmp
R=$PWD
cd /tmp
A="--algo AES256-GCM-HMAC-SHA256 --reps 3"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$OUT/trace -o run --output-format csv -- python3 $R/tools/crypt_bench.py $A > $R/$OUT/trace.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU -d $R/$OUT/sq -o run --output-format csv -- python3 $R/tools/crypt_bench.py $A > $R/$OUT/sq.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM -d $R/$OUT/sq2 -o run --output-format csv -- python3 $R/tools/crypt_bench.py $A > $R/$OUT/sq2.log 2>&1 || exit 1
