set -o pipefail
mkdir -p gpurun_out/v47
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --cpu-sample 0 --batch 4096 > gpurun_out/v47/bench_b4096.log 2>&1 && \
timeout -k 10 500 python -u bench.py --cpu-sample 0 --batch 8192 --steps 1 > gpurun_out/v47/bench_b8192.log 2>&1
