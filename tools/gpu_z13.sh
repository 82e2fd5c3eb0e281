#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/z13
timeout -k 10 300 python3 -u tools/zdiag.py gpurun_out/z13 > gpurun_out/z13/diag.log 2>&1
rc=$?; tail -1 gpurun_out/z13/diag.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_z12.sh
