set -o pipefail
mkdir -p gpurun_out
SVS_POA_TRACE=gpurun_out/v29_bench_trace.txt timeout -k 10 900 python -u bench.py > gpurun_out/v29_bench_default.log 2>&1
