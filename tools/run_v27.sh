set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_poa_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_v27.log 2>&1 && \
timeout -k 10 200 python -u tools/poa_probe.py --windows 2048 --check 2 > gpurun_out/v27_probe2048.log 2>&1 && \
SVS_POA_PRUNE_SLACK=100 timeout -k 10 200 python -u tools/poa_probe.py --windows 2048 > gpurun_out/v27_probe2048_allalive.log 2>&1 && \
SVS_POA_PRUNE_SLACK=0.01 SVS_POA_TRACE=gpurun_out/v27_trace.txt timeout -k 10 200 python -u tools/poa_probe.py --windows 2048 > gpurun_out/v27_probe2048_s001.log 2>&1
