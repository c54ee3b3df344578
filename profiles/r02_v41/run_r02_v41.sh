set -o pipefail
# Export kernel chain-row test from the chunk's edge registers (lane shuffle)
# instead of a dependent global load (r02_v40: the load made the export
# kernel slower, 572 vs 500 ms). A/B on the MSA probe against r02_v38.
D=gpurun_out/r02_v41
mkdir -p $D
export TMPDIR=/tmp
V=$PWD/svscope_amd/lib/variants
p() { timeout -k 10 200 python -u tools/poa_probe.py --windows 2048 > $D/probe_$1.log 2>&1; }
timeout -k 10 400 python -u -m pytest tests/test_poa_gpu.py tests/test_decision_gpu.py -x -v --timeout 240 --timeout-method thread > $D/pytest_poa.log 2>&1 && \
SVS_LIB_PATH=$V/libsvscope_hip_v38.so p v38a && p new1 && SVS_LIB_PATH=$V/libsvscope_hip_v38.so p v38b && p new2
