#!/bin/bash
# One documented driver for GPU sessions (run from the repo root through gpurun); every step
# writes under gpurun_out/<OUT>/ and the script stops at the first failing step.
#
#   tools/gpu_session.sh OUT step [step ...]
#
# steps:
#   suite            pytest -m gpu (thread timeouts), then smoke()
#   tests:PATTERN    pytest -m gpu -k PATTERN (e.g. tests:writer)
#   bench            the driver's default line: bench.py --gpus 1 --steps 20 --warmup 5
#   bench:ARGS       bench.py with ARGS (commas for spaces: bench:--config,4)
#   prof             the default bench line under rocprofv3 --kernel-trace --stats, then its
#                    FETCH_SIZE pass (separate runs: no PMC with tracing)
#   prof:TAG:ARGS    the same for bench.py ARGS (commas for spaces), files named TAG_*
#   kbench:ARGS      tools/kbench.py ARGS (same-process A/B of build/variants/*.so)
#   writer:ARGS      build/writer_bench ARGS (commas for spaces)
#   writerpin:CPUS:ARGS  the same under taskset -c CPUS (threads confined to the CPU quota)
#   valu:ARGS        build/valu_rate ARGS (tools/valu_rate.hip: the VALU rate table, or "rk": the
#                    Rabin-Karp hot loop alone over config 2's bytes)
#   sq:TAG:ARGS      SQ counters (VALU/LDS/wait) of bench.py ARGS, one --pmc pass
#   trace:ARGS       tools/trace_pipe.py build/libkcdc_trace.so ARGS (per-wave timeline of the batch kernel)
#   cprof:NAME:KIND  rocprofv3 --kernel-trace --stats of compress_bench.py --name NAME --only KIND (per-kernel time)
#   probe:ARGS       tools/batch_probe.py ARGS (one bounded launch: queue stats, mismatched streams;
#                    PROBE_REPS=n repeats the launch until one loses a stream)
#   vprobe:V:ARGS    the same with build/variants/libkcdc_V.so
#   compress:NAMES   tools/compress_bench.py --gib 4 for each compressor name (commas between names)
set -u
OUT=gpurun_out/${1:?usage: tools/gpu_session.sh OUT step...}
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
args() { echo "${1//,/ }"; }
for step in "$@"; do
  echo "== $step $(date +%T)"
  case "$step" in
    suite)
      timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/suite.log" 2>&1
      rc=$?; tail -3 "$OUT/suite.log"; [ $rc -eq 0 ] || exit $rc
      timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
      tail -1 "$OUT/smoke.log" ;;
    tests:*)
      k=${step#tests:}
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -k "$k" --timeout 200 --timeout-method thread > "$OUT/tests_$k.log" 2>&1
      rc=$?; tail -3 "$OUT/tests_$k.log"; [ $rc -eq 0 ] || exit $rc ;;
    bench)
      timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || exit $?
      tail -c 600 "$OUT/bench_default.json" ;;
    bench:*)
      a=$(args "${step#bench:}"); t=$(echo "$a" | tr -c 'A-Za-z0-9' '_')
      timeout -k 10 400 python -u bench.py $a > "$OUT/bench_$t.json" 2> "$OUT/bench_$t.err" || exit $?
      tail -c 600 "$OUT/bench_$t.json" ;;
    prof|prof:*)
      if [ "$step" = prof ]; then tag=default; a="--gpus 1 --steps 20 --warmup 5"; else
        r=${step#prof:}; tag=${r%%:*}; a=$(args "${r#*:}"); fi
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/${tag}_trace" -o run --output-format csv -- python3 bench.py $a > "$OUT/${tag}_trace.json" 2> "$OUT/${tag}_trace.err" || exit $?
      timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE -d "$OUT/${tag}_fetch" -o run --output-format csv -- python3 bench.py $a > "$OUT/${tag}_fetch.json" 2> "$OUT/${tag}_fetch.err" || exit $?
      echo "profiled $tag" ;;
    sq:*)
      r=${step#sq:}; tag=${r%%:*}; a=$(args "${r#*:}")
      timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU -d "$OUT/${tag}_sq" -o run --output-format csv -- python3 bench.py $a > "$OUT/${tag}_sq.json" 2> "$OUT/${tag}_sq.err" || exit $?
      echo "counted $tag" ;;
    kbench:*)
      a=$(args "${step#kbench:}"); t=$(echo "$a" | tr -c 'A-Za-z0-9' '_')
      timeout -k 10 300 python -u tools/kbench.py $a > "$OUT/kbench_$t.log" 2>&1 || exit $?
      grep -A3 '"prod"' "$OUT/kbench_$t.log" | head -4 ;;
    writer:*)
      a=$(args "${step#writer:}"); t=$(echo "$a" | tr -c 'A-Za-z0-9' '_')
      timeout -k 10 300 ./build/writer_bench $a > "$OUT/writer_$t.json" 2> "$OUT/writer_$t.err" || exit $?
      cat "$OUT/writer_$t.json" ;;
    writerpin:*)
      r=${step#writerpin:}; cpus=${r%%:*}; a=$(args "${r#*:}"); t=$(echo "$cpus $a" | tr -c 'A-Za-z0-9' '_')
      timeout -k 10 300 taskset -c "$cpus" ./build/writer_bench $a > "$OUT/writerpin_$t.json" 2> "$OUT/writerpin_$t.err" || exit $?
      cat "$OUT/writerpin_$t.json" ;;
    valu:*)
      a=$(args "${step#valu:}"); t=$(echo "$a" | tr -c 'A-Za-z0-9' '_')
      timeout -k 10 300 ./build/valu_rate $a > "$OUT/valu_$t.log" 2>&1 || exit $?
      tail -4 "$OUT/valu_$t.log" ;;
    trace:*)
      a=$(args "${step#trace:}"); t=$(echo "$a" | tr -c 'A-Za-z0-9' '_')
      timeout -k 10 300 python -u tools/trace_pipe.py build/libkcdc_trace.so $a > "$OUT/trace_$t.log" 2>&1 || exit $?
      tail -12 "$OUT/trace_$t.log" ;;
    cprof:*)
      r=${step#cprof:}; nm=${r%%:*}; kind=${r#*:}
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/cprof_${nm}_$kind" -o run --output-format csv -- python3 tools/compress_bench.py --gib 4 --iters 3 --name "$nm" --only "$kind" > "$OUT/cprof_${nm}_$kind.log" 2>&1 || exit $?
      echo "profiled $nm $kind" ;;
    vprobe:*)
      r=${step#vprobe:}; v=${r%%:*}; a=$(args "${r#*:}"); t=$(echo "$v $a" | tr -c 'A-Za-z0-9' '_')
      KCDC_ALLOW_VARIANT_LIB=1 KCDC_LIB=build/variants/libkcdc_$v.so timeout -k 10 240 python -u tools/batch_probe.py $a > "$OUT/vprobe_$t.log" 2>&1 || { cat "$OUT/vprobe_$t.log"; exit 1; }
      cat "$OUT/vprobe_$t.log" ;;
    probe:*)
      a=$(args "${step#probe:}"); t=$(echo "$a" | tr -c 'A-Za-z0-9' '_')
      timeout -k 10 240 python -u tools/batch_probe.py $a > "$OUT/probe_$t.log" 2>&1 || { cat "$OUT/probe_$t.log"; exit 1; }
      cat "$OUT/probe_$t.log" ;;
    compress:*)
      for nm in $(args "${step#compress:}"); do
        timeout -k 10 300 python -u tools/compress_bench.py --gib 4 --iters 3 --name "$nm" > "$OUT/compress_$nm.log" 2>&1 || exit $?
        tail -1 "$OUT/compress_$nm.log" | cut -c1-400
      done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "session done"
