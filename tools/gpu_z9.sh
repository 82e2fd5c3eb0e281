#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/z9
KCDC_LIB=build/variants/libkcdc_rankonly.so KCDC_ALLOW_VARIANT_LIB=1 timeout -k 10 300 python3 -u tools/ztrace.py 64 deflate-default > gpurun_out/z9/rankonly.json 2> gpurun_out/z9/err.log
rc=$?; cat gpurun_out/z9/rankonly.json; exit $rc
