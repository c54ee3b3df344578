set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_v32.log 2>&1 && \
timeout -k 10 200 python -u tools/poa_probe.py --windows 2048 --check 2 > gpurun_out/v32_probe2048.log 2>&1 && \
SVS_POA_TRACE=gpurun_out/v32_bench_trace.txt timeout -k 10 900 python -u bench.py > gpurun_out/v32_bench_default.log 2>&1
