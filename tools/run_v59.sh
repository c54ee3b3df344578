set -o pipefail
mkdir -p gpurun_out/v59
export TMPDIR=/tmp
timeout -k 10 500 python -u bench.py --cpu-sample 0 --batch 6144 > gpurun_out/v59/bench_b6144.log 2>&1 && \
timeout -k 10 500 python -u bench.py --cpu-sample 0 --batch 4096 > gpurun_out/v59/bench_b4096.log 2>&1 && \
timeout -k 10 600 python -u bench.py --cpu-sample 0 --batch 8192 > gpurun_out/v59/bench_b8192.log 2>&1
