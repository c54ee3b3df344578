set -o pipefail
mkdir -p gpurun_out
for v in base occ6 occ7; do
  echo "== $v" >> gpurun_out/v33_occ.log
  if [ $v = base ]; then unset SVS_LIB_PATH; else export SVS_LIB_PATH=$PWD/svscope_amd/lib/variants/libsvscope_hip_$v.so; fi
  timeout -k 10 200 python -u tools/poa_probe.py --windows 2048 --check 1 >> gpurun_out/v33_occ.log 2>&1 || exit 1
done
