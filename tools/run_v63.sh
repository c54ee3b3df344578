set -o pipefail
mkdir -p gpurun_out/v63
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/v63/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/v63/smoke.log 2>&1 && \
timeout -k 10 900 python -u bench.py > gpurun_out/v63/bench_default.log 2>&1 && \
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/v63/bench_ktrace -o run -- python3 bench.py --cpu-sample 0 > gpurun_out/v63/bench_under_rocprof.log 2>&1
