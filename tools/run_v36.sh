set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_poa_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_v36.log 2>&1 && \
timeout -k 10 200 python -u tools/poa_probe.py --windows 2048 --check 1 > gpurun_out/v36_probe.log 2>&1 && \
SVS_LIB_PATH=$PWD/svscope_amd/lib/variants/libsvscope_hip_occ6.so timeout -k 10 200 python -u tools/poa_probe.py --windows 2048 --check 1 > gpurun_out/v36_probe_occ6.log 2>&1
