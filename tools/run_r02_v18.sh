set -o pipefail
D=gpurun_out/r02_v18
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $D/pytest_gpu.log 2>&1 && \
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench_driver_cmd.log 2>&1 && \
timeout -k 10 300 python -u tools/prune_probe.py --windows 512 --error 0.08 --ins-min 200 --ins-max 801 --check 1 > $D/prune_default.log 2>&1 && \
timeout -k 10 400 python -u tools/prune_probe.py --windows 512 --check 2 > $D/prune_harsh.log 2>&1 && \
SVS_POA_TRACE=$D/trace_b512.txt timeout -k 10 300 python -u bench.py --steps 6 --warmup 1 --cpu-sample 0 > $D/bench_trace.log 2>&1
