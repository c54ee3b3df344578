set -o pipefail
mkdir -p gpurun_out/r06_s1
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_poa_gpu.py tests/test_decision_gpu.py -x -v --timeout 240 --timeout-method thread > gpurun_out/r06_s1/pytest.log 2>&1 || { tail -40 gpurun_out/r06_s1/pytest.log; exit 1; }
tail -2 gpurun_out/r06_s1/pytest.log
AB_STEPS=20 AB_WARMUP=5 bash tools/ab_bench.sh r06_s1 'base SVS_POA_FOLD_WORKERS=0' 'stream SVS_POA_FOLD_WORKERS=256' 'base2 SVS_POA_FOLD_WORKERS=0' 'stream2 SVS_POA_FOLD_WORKERS=256'
