set -o pipefail
D=gpurun_out/r05_a2; mkdir -p $D; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_poa_gpu.py -x -v --timeout 120 --timeout-method thread > $D/pytest_poa.log 2>&1 || { tail -30 $D/pytest_poa.log; exit 1; }
tail -2 $D/pytest_poa.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { tail -30 $D/pytest_gpu.log; exit 1; }
tail -2 $D/pytest_gpu.log
AB_STEPS=20 AB_WARMUP=5 bash tools/ab_bench.sh r05_a2 'new' 'base SVS_LIB_PATH=svscope_amd/lib/variants/libsvscope_hip_base.so'
