set -o pipefail
# A/B on the MSA probe: v36 = r02_v36 product, product = + 32-bit byte
# offsets for the row-record / carry loads and carry stores, fixed = product
# with spoa's default scores as compile-time constants (SVS_FIXED_SCORES)
D=gpurun_out/r02_v37
mkdir -p $D
export TMPDIR=/tmp
V=$PWD/svscope_amd/lib/variants
p() { timeout -k 10 200 python -u tools/poa_probe.py --windows 2048 > $D/probe_$1.log 2>&1; }
timeout -k 10 400 python -u -m pytest tests/test_poa_gpu.py tests/test_decision_gpu.py -x -v --timeout 240 --timeout-method thread > $D/pytest_poa.log 2>&1 && \
SVS_LIB_PATH=$V/libsvscope_hip_v36.so p v36a && p new1 && SVS_LIB_PATH=$V/libsvscope_hip_fixed.so p fixed1 && \
SVS_LIB_PATH=$V/libsvscope_hip_v36.so p v36b && p new2 && SVS_LIB_PATH=$V/libsvscope_hip_fixed.so p fixed2
