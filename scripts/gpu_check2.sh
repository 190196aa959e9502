set -o pipefail
mkdir -p gpurun_out/v2
ASAN_OPTIONS=detect_leaks=0 timeout -k 10 180 ./build/abi_asan > gpurun_out/v2/abi_asan.log 2>&1; echo ASAN_RC=$?; tail -1 gpurun_out/v2/abi_asan.log
for i in 1 2; do timeout -k 10 120 ./build/abi_so 2>&1 | tail -1; done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/v2/pytest_gpu.log 2>&1; echo PYTEST_RC=$?; tail -2 gpurun_out/v2/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/v2/bench_config3.json 2> gpurun_out/v2/e0; echo BENCH_RC=$?; cut -c1-300 gpurun_out/v2/bench_config3.json
timeout -k 10 300 python bench.py --config subband --no-cpu-baseline > gpurun_out/v2/bench_subband.json 2> gpurun_out/v2/e1; echo SUB_RC=$?; cut -c1-300 gpurun_out/v2/bench_subband.json
