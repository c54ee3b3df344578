set -o pipefail
D=gpurun_out/r02_v4
mkdir -p $D
export TMPDIR=/tmp
for cfg in "base:" "wpj6:SVS_POA_WPJ=6" "resident:SVS_POA_WPJ_RESIDENT=1" "act768:SVS_POA_ACTIVE_JOBS=768" "wpj5:SVS_POA_WPJ=5" "act1536w4:SVS_POA_ACTIVE_JOBS=1536 SVS_POA_WPJ=4"; do
  name=${cfg%%:*}; envs=${cfg#*:}
  env $envs timeout -k 10 200 python -u tools/poa_probe.py --windows 2048 > $D/probe_$name.log 2>&1 || exit 1
done
