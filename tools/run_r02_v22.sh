set -o pipefail
D=gpurun_out/r02_v22
mkdir -p $D
export TMPDIR=/tmp
p() { timeout -k 10 200 python -u tools/poa_probe.py --windows 2048 > $D/probe_$1.log 2>&1; }
p base && SVS_POA_ACTIVE_JOBS=1280 p act1280 && SVS_POA_ACTIVE_JOBS=1536 p act1536 && SVS_POA_WPJ=4 p wpj4 && \
SVS_POA_ACTIVE_JOBS=1536 SVS_POA_WPJ=4 p act1536w4 && SVS_POA_ACTIVE_JOBS=768 p act768 && p base2
