set -o pipefail
D=gpurun_out/r02_v10
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 120 ./tools/microbench/issue_rates > $D/issue_rates.log 2>&1 || exit 1
for v in base carry all3; do
  if [ $v = base ]; then unset SVS_LIB_PATH; else export SVS_LIB_PATH=$PWD/svscope_amd/lib/variants/libsvscope_hip_$v.so; fi
  timeout -k 10 200 python -u tools/poa_probe.py --windows 2048 --check 1 > $D/probe_$v.log 2>&1 || exit 1
done
