set -o pipefail
mkdir -p gpurun_out/r06_u1
export TMPDIR=/tmp
V=svscope_amd/lib/variants/libsvscope_hip_us.so
SVS_LIB_PATH=$V timeout -k 10 600 python -u -m pytest tests/test_poa_gpu.py -x -v --timeout 240 --timeout-method thread -k "variants or handoff or handcheck" > gpurun_out/r06_u1/pytest.log 2>&1 || { tail -40 gpurun_out/r06_u1/pytest.log; exit 1; }
tail -2 gpurun_out/r06_u1/pytest.log
AB_STEPS=20 AB_WARMUP=5 bash tools/ab_bench.sh r06_u1 'base' "us SVS_LIB_PATH=$V" 'base2' "us2 SVS_LIB_PATH=$V"
for f in gpurun_out/r06_u1/b_*.json; do python3 -c "import json;d=json.load(open('$f'));b=d['breakdown'];print('$f', b['dp_end_to_launch_done_ms'], b['poa_launches'], round(b['dp_end_to_launch_done_ms']/b['poa_launches'],2), b['em_kernel_s'], d['roofline']['busy_ms'])"; done
