set -o pipefail
# A/B on the MSA probe: base = r02_v35 kernel (SVS_ROWTAIL_OLD), product =
# scalar publish countdown (all lanes store), per-lane sink maximum behind a
# scalar branch, lanes past L folded into ub, 32-bit code offsets;
# carryall = product + carry stores from every lane
D=gpurun_out/r02_v36
mkdir -p $D
export TMPDIR=/tmp
V=$PWD/svscope_amd/lib/variants
p() { timeout -k 10 200 python -u tools/poa_probe.py --windows 2048 > $D/probe_$1.log 2>&1; }
timeout -k 10 400 python -u -m pytest tests/test_poa_gpu.py tests/test_decision_gpu.py -x -v --timeout 240 --timeout-method thread > $D/pytest_poa.log 2>&1 && \
SVS_LIB_PATH=$V/libsvscope_hip_base.so p base1 && p new1 && SVS_LIB_PATH=$V/libsvscope_hip_carryall.so p carryall1 && \
SVS_LIB_PATH=$V/libsvscope_hip_base.so p base2 && p new2 && SVS_LIB_PATH=$V/libsvscope_hip_carryall.so p carryall2
