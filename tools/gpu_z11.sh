#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/z11
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_compress.py -k "s2" > gpurun_out/z11/t.log 2>&1
rc=$?; tail -4 gpurun_out/z11/t.log; exit $rc
