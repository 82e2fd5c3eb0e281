#!/bin/bash
# round 6 (late): where 1024 x 16 MiB loses against 4096 x 4 MiB -- per-wave trace and knobs
set -o pipefail
O=gpurun_out/s6j; mkdir -p $O
timeout -k 10 120 python3 -u tools/trace_pipe.py build/libkcdc_trace.so 1024 16 > $O/trace_1024_16.json 2> $O/err.log || exit 1
timeout -k 10 120 python3 -u tools/trace_pipe.py build/libkcdc_trace.so 4096 4 > $O/trace_4096_4.json 2>> $O/err.log || exit 1
timeout -k 10 200 python3 -u tools/kbench.py --streams 1024 --mib 16 --glob 'none' --knob 6=1 --knob 6=2 --knob 8=1024 --knob 8=4096 --rounds 5 > $O/kb_1024_16.log 2>> $O/err.log || exit 1
cat $O/kb_1024_16.log | tail -40
