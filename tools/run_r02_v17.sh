set -o pipefail
D=gpurun_out/r02_v17
mkdir -p $D
export TMPDIR=/tmp
p() { timeout -k 10 200 python -u tools/poa_probe.py --windows 2048 > $D/probe_$1.log 2>&1; }
export SVS_POA_PRUNE_MAX_RETRIES=16 SVS_POA_PRUNE_RETRY_SLACK=0.1
SVS_POA_PRUNE_SLACK=0.05 p s05 && \
SVS_POA_PRUNE_SLACK=0.03 p s03 && \
SVS_POA_PRUNE_SLACK=0.03 SVS_POA_PRUNE_ADAPT=2 p s03a2 && \
SVS_POA_PRUNE_SLACK=0.02 SVS_POA_PRUNE_ADAPT=2 p s02a2 && \
SVS_POA_PRUNE_SLACK=0.025 SVS_POA_PRUNE_ADAPT=1.5 p s025a15 && \
SVS_POA_PRUNE_SLACK=0.04 p s04
