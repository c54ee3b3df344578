set -o pipefail
mkdir -p gpurun_out/r06_w1
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_poa_gpu.py -x -v --timeout 240 --timeout-method thread > gpurun_out/r06_w1/pytest.log 2>&1 || { tail -40 gpurun_out/r06_w1/pytest.log; exit 1; }
tail -2 gpurun_out/r06_w1/pytest.log
V=svscope_amd/lib/variants
AB_STEPS=20 AB_WARMUP=5 bash tools/ab_bench.sh r06_w1 "head SVS_LIB_PATH=$V/libsvscope_hip_head.so" 'both' "waitonly SVS_LIB_PATH=$V/libsvscope_hip_waitonly.so" "head2 SVS_LIB_PATH=$V/libsvscope_hip_head.so" 'both2' "waitonly2 SVS_LIB_PATH=$V/libsvscope_hip_waitonly.so"
