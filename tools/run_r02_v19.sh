set -o pipefail
D=gpurun_out/r02_v19
mkdir -p $D
export TMPDIR=/tmp
b() { timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-sample 0 "${@:2}" > $D/bench_$1.log 2>&1; }
OLD="SVS_POA_PRUNE_SLACK=0.05 SVS_POA_PRUNE_ADAPT=1 SVS_POA_PRUNE_RETRY_SLACK=none SVS_POA_PRUNE_MAX_RETRIES=2"
env $OLD bash -c "$(declare -f b); D=$D b old1" && \
b new1 && \
b new_d8 --depth 8 && \
env $OLD bash -c "$(declare -f b); D=$D b old2" && \
b new2 && \
b new_d6 --depth 6
