# round 6: RK lane multiplier A/B, the round-6 RK kernel's trace/FETCH/SQ passes, the writer tests
# after the lifetime fixes, writer finish latency
set -o pipefail
O=gpurun_out/s6e; mkdir -p $O
for nm in DYNAMIC-4M-RABINKARP DYNAMIC-1M-RABINKARP DYNAMIC-128K-RABINKARP; do
  timeout -k 10 300 python -u tools/kbench.py --name $nm --rounds 7 > $O/kb_$nm.log 2>&1 || exit 1
done
A="--splitter DYNAMIC-4M-RABINKARP --steps 10 --warmup 3 --no-cpu-baseline --no-host-inclusive --no-hash --pipeline-slots 0 --no-encrypt"
tools/profile_configs.sh $O rk "$A" && tools/profile_sq.sh $O rk "$A" || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k writer --timeout 200 --timeout-method thread > $O/tests_writer.log 2>&1 || { tail -20 $O/tests_writer.log; exit 1; }
tail -2 $O/tests_writer.log
for h in none BLAKE2B-256-128 BLAKE3-256-128; do
  timeout -k 10 300 ./build/writer_bench 32 512 64 DYNAMIC-4M-BUZHASH 256 3 $h > $O/writer_32_512_$h.json 2> $O/writer_32_512_$h.err || exit 1
  cat $O/writer_32_512_$h.json
done
