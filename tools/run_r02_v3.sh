set -o pipefail
D=gpurun_out/r02_v3
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_poa_gpu.py tests/test_tdscope_gpu.py -x -v --timeout 240 --timeout-method thread > $D/pytest_poa_tdscope.log 2>&1 && \
SVS_LIB_PATH=$PWD/svscope_amd/lib/variants/libsvscope_hip_prof.so SVS_STRIP_PROF=1 timeout -k 10 300 python -u tools/poa_probe.py --windows 2048 > $D/probe_prof.log 2>&1 && \
timeout -k 10 300 python -u tools/poa_probe.py --windows 2048 > $D/probe.log 2>&1
