# Long path on the GPU box: parity tests, then config 3 (16 GiB) with the product build and a
# variant (build/variants/libkcdc_$1.so), then the `kopia benchmark splitter` defaults.
set -e
V=${1:-serres}
mkdir -p gpurun_out/c3ab
timeout -k 10 400 python -u -m pytest tests/test_gpu_long.py tests/test_gpu_files.py -x -v --timeout 200 --timeout-method thread > gpurun_out/c3ab/pytest.log 2>&1
timeout -k 10 120 python -u bench.py --config 3 --long-gib 16 --steps 5 > gpurun_out/c3ab/new.json 2>/dev/null
timeout -k 10 120 python -u -c "import sys; import kopia_amd._lib as L; L.LIB_PATH='build/variants/libkcdc_$V.so'; sys.argv=['bench.py','--config','3','--long-gib','16','--steps','5']; import bench; bench.main()" > gpurun_out/c3ab/old.json 2>/dev/null
timeout -k 10 120 python -u -m kopia_amd.benchmark_splitters > gpurun_out/c3ab/bench_default.txt 2>&1
timeout -k 10 120 python -u -m kopia_amd.benchmark_splitters --data-size 256MiB --block-count 1 > gpurun_out/c3ab/bench_config1.txt 2>&1
