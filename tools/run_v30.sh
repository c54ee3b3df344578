set -o pipefail
mkdir -p gpurun_out
for cfg in "SVS_POA_WPJ=4" "SVS_POA_WPJ=2" "SVS_POA_WPJ=16" "SVS_POA_ACTIVE_JOBS=2048 SVS_POA_WPJ=4" "SVS_POA_ACTIVE_JOBS=2048 SVS_POA_WPJ=2"; do
  echo "== $cfg" >> gpurun_out/v30_sweep.log
  env $cfg timeout -k 10 200 python -u tools/poa_probe.py --windows 2048 >> gpurun_out/v30_sweep.log 2>&1 || exit 1
done
