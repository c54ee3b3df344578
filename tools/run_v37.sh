set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_v37.log 2>&1 && \
SVS_POA_TRACE=gpurun_out/v37_bench_trace.txt timeout -k 10 900 python -u bench.py > gpurun_out/v37_bench_default.log 2>&1
