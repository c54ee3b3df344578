set -o pipefail
mkdir -p gpurun_out/r06_q1
export TMPDIR=/tmp
AB_STEPS=20 AB_WARMUP=5 bash tools/ab_bench.sh r06_q1 'base' 'crit SVS_POA_QUEUE_ORDER=1' 'coarse SVS_POA_QUEUE_ORDER=2' 'base2' 'crit2 SVS_POA_QUEUE_ORDER=1' 'coarse2 SVS_POA_QUEUE_ORDER=2'
