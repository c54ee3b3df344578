set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_poa_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_v26.log 2>&1 && \
timeout -k 10 200 python -u tools/poa_probe.py --windows 2048 --check 2 > gpurun_out/v26_probe2048.log 2>&1 && \
SVS_POA_PRUNE=0 timeout -k 10 200 python -u tools/poa_probe.py --windows 2048 > gpurun_out/v26_probe2048_noprune.log 2>&1
