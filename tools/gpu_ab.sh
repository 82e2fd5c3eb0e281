#!/bin/bash
# One GPU call: GPU parity suite, variant A/B timing, SQ counter passes on the bench.
#   usage: tools/gpu_ab.sh TAG [skip-tests]
set -u
TAG=${1:-ab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "${2:-}" != "skip-tests" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -3 $OUT/pytest_gpu.log
fi
timeout -k 10 300 python -u tools/kbench.py --rounds 5 --reps 5 > $OUT/kbench.log 2>&1 || { tail -30 $OUT/kbench.log; exit 1; }
cat $OUT/kbench.log
[ "${3:-}" = "nopmc" ] && exit 0
for pass in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
            "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE GRBM_COUNT"; do
  n=$(echo $pass | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $pass -d $OUT/pmc_$n -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-inclusive > $OUT/pmc_$n.log 2>&1 || { tail -20 $OUT/pmc_$n.log; exit 1; }
done
echo done
