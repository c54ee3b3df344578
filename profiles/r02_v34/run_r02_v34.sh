set -o pipefail
# A/B on the MSA probe: base = export-kernel register windows (prepwin),
# pub = + publish countdown, product = + lane-0 buffer-store carries
D=gpurun_out/r02_v34
mkdir -p $D
export TMPDIR=/tmp
V=$PWD/svscope_amd/lib/variants
p() { timeout -k 10 200 python -u tools/poa_probe.py --windows 2048 > $D/probe_$1.log 2>&1; }
timeout -k 10 400 python -u -m pytest tests/test_poa_gpu.py tests/test_decision_gpu.py -x -v --timeout 240 --timeout-method thread > $D/pytest_poa.log 2>&1 && \
SVS_LIB_PATH=$V/libsvscope_hip_prepwin.so p base1 && SVS_LIB_PATH=$V/libsvscope_hip_pub.so p pub1 && p pubcarry1 && \
SVS_LIB_PATH=$V/libsvscope_hip_prepwin.so p base2 && SVS_LIB_PATH=$V/libsvscope_hip_pub.so p pub2 && p pubcarry2
