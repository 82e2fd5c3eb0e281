#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/z5
KCDC_LIB=build/libkcdc_trace.so KCDC_ALLOW_VARIANT_LIB=1 timeout -k 10 300 python3 -u tools/ztrace.py 64 > gpurun_out/z5/trace.json 2> gpurun_out/z5/err.log
rc=$?; tail -22 gpurun_out/z5/trace.json; exit $rc
