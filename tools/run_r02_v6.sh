set -o pipefail
D=gpurun_out/r02_v6
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_aln_feature_gpu.py -x -v --timeout 240 --timeout-method thread > $D/pytest_alnfeature.log 2>&1 || exit 1
for v in base pf23 occ7 occ8 occ5; do
  if [ $v = base ]; then unset SVS_LIB_PATH; else export SVS_LIB_PATH=$PWD/svscope_amd/lib/variants/libsvscope_hip_$v.so; fi
  timeout -k 10 200 python -u tools/poa_probe.py --windows 2048 --check 2 > $D/probe_$v.log 2>&1 || exit 1
done
