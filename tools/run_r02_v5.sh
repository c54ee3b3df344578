set -o pipefail
D=gpurun_out/r02_v5
mkdir -p $D
export TMPDIR=/tmp
for v in base salu40 valu40 valu80; do
  if [ $v = base ]; then unset SVS_LIB_PATH; else export SVS_LIB_PATH=$PWD/svscope_amd/lib/variants/libsvscope_hip_$v.so; fi
  timeout -k 10 200 python -u tools/poa_probe.py --windows 2048 > $D/probe_$v.log 2>&1 || exit 1
done
