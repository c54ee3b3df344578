set -o pipefail
mkdir -p gpurun_out/v42
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/v42/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/v42/smoke.log 2>&1 && \
timeout -k 10 900 python -u bench.py > gpurun_out/v42/bench_default.log 2>&1
