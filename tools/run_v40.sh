set -o pipefail
mkdir -p gpurun_out/v40
export TMPDIR=/tmp
timeout -k 10 300 env SVS_POA_STREAMS=2 python -u bench.py --cpu-sample 0 > gpurun_out/v40/bench_2streams.log 2>&1 && \
timeout -k 10 300 env SVS_POA_STREAMS=1 python -u bench.py --cpu-sample 0 > gpurun_out/v40/bench_1stream.log 2>&1
