set -o pipefail
mkdir -p gpurun_out/r06_c1
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_em_gpu.py tests/test_decision_gpu.py -x -v --timeout 240 --timeout-method thread -k "em or reference" > gpurun_out/r06_c1/pytest.log 2>&1 || { tail -40 gpurun_out/r06_c1/pytest.log; exit 1; }
tail -2 gpurun_out/r06_c1/pytest.log
AB_STEPS=20 AB_WARMUP=5 bash tools/ab_bench.sh r06_c1 'base' 'emold SVS_LIB_PATH=svscope_amd/lib/variants/libsvscope_hip_emkc15.so' 'fold16 SVS_POA_FOLD_CUS=16' 'fold32 SVS_POA_FOLD_CUS=32' 'base2' 'emold2 SVS_LIB_PATH=svscope_amd/lib/variants/libsvscope_hip_emkc15.so'
for f in gpurun_out/r06_c1/b_*.json; do python3 -c "import json;d=json.load(open('$f'));b=d['breakdown'];print('$f', b['dp_end_to_launch_done_ms'], b['poa_launches'], round(b['dp_end_to_launch_done_ms']/b['poa_launches'],2), b['em_kernel_s'], d['roofline']['busy_ms'])"; done
