#!/bin/bash
# zstd block split: ratio and phases per segment weight
set -o pipefail
mkdir -p gpurun_out/z14
for W in 0 16 48 1000; do
KCDC_LIB=build/variants/libkcdc_w$W.so KCDC_ALLOW_VARIANT_LIB=1 timeout -k 10 300 python3 -u tools/ztrace.py 64 > gpurun_out/z14/w$W.json 2> gpurun_out/z14/err.log || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/z14/w$W.json')); print($W, d['ratio'], d['total_cycles_mean'], d['fse pass']['mean'])"
done
