set -o pipefail
D=gpurun_out/r02_v16
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_poa_gpu.py -x -v --timeout 120 --timeout-method thread -k "variants or pruning" > $D/pytest_poa.log 2>&1 || exit 1
p() { timeout -k 10 200 python -u tools/poa_probe.py --windows 2048 > $D/probe_$1.log 2>&1; }
SVS_POA_PRUNE_RETRY_SLACK=none p old05 && \
p s05 && \
SVS_POA_PRUNE_SLACK=0.03 p s03 && \
SVS_POA_PRUNE_SLACK=0.02 p s02 && \
SVS_POA_PRUNE_SLACK=0.03 SVS_POA_PRUNE_MAX_RETRIES=16 p s03m16 && \
SVS_POA_PRUNE_SLACK=0.02 SVS_POA_PRUNE_MAX_RETRIES=16 p s02m16 && \
SVS_POA_PRUNE_SLACK=0.02 SVS_POA_PRUNE_MAX_RETRIES=16 SVS_POA_PRUNE_RETRY_SLACK=0.1 p s02m16r10
