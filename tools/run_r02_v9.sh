set -o pipefail
D=gpurun_out/r02_v9
mkdir -p $D
export TMPDIR=/tmp
for v in base fixed code fixcode; do
  if [ $v = base ]; then unset SVS_LIB_PATH; else export SVS_LIB_PATH=$PWD/svscope_amd/lib/variants/libsvscope_hip_$v.so; fi
  timeout -k 10 200 python -u tools/poa_probe.py --windows 2048 --check 2 > $D/probe_$v.log 2>&1 || exit 1
done
export SVS_LIB_PATH=$PWD/svscope_amd/lib/variants/libsvscope_hip_fixcode.so
timeout -k 10 400 python -u -m pytest tests/test_poa_gpu.py -x -q --timeout 240 --timeout-method thread > $D/pytest_poa_fixcode.log 2>&1
