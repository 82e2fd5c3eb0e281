#!/bin/bash
# SQ/LDS counter passes (one rocprofv3 --pmc run each) over a bench command.
# usage: tools/profile_sq.sh OUTDIR TAG "bench args"
set -u
OUT=$1; TAG=$2; ARGS=$3
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for pass in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
            "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pass -d "$OUT/${TAG}_sq$i" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/${TAG}_sq$i.log" 2>&1 || exit $?
done
echo done
