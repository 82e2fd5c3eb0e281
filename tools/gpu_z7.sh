#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/z7
KCDC_LIB=build/libkcdc_trace.so KCDC_ALLOW_VARIANT_LIB=1 timeout -k 10 300 python3 -u tools/ztrace.py 64 deflate-default > gpurun_out/z7/deflate.json 2> gpurun_out/z7/err.log
rc=$?; cat gpurun_out/z7/deflate.json; exit $rc
