set -o pipefail
mkdir -p gpurun_out/v52
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_misscore_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/v52/pytest_misscore.log 2>&1 && \
timeout -k 10 300 python -u tools/misscore_probe.py --pairs 4096 > gpurun_out/v52/ms_probe.log 2>&1 && \
timeout -k 10 300 env SVS_MS_TB=lane python -u tools/misscore_probe.py --pairs 4096 --cpu-sample 0 > gpurun_out/v52/ms_probe_lane.log 2>&1
