#!/bin/bash
# zstd_emit_kernel phase times (KCDC_TRACE build)
set -o pipefail
mkdir -p gpurun_out/z3
KCDC_LIB=build/libkcdc_trace.so KCDC_ALLOW_VARIANT_LIB=1 timeout -k 10 300 python3 -u tools/ztrace.py 64 > gpurun_out/z3/trace.json 2> gpurun_out/z3/err.log
rc=$?; cat gpurun_out/z3/trace.json; tail -3 gpurun_out/z3/err.log; exit $rc
