set -o pipefail
mkdir -p gpurun_out/r06_q2
export TMPDIR=/tmp
AB_STEPS=20 AB_WARMUP=5 bash tools/ab_bench.sh r06_q2 'base' 'c4 SVS_POA_QUEUE_ORDER=2' 'c8 SVS_POA_QUEUE_ORDER=3' 'c2 SVS_POA_QUEUE_ORDER=4' 'base2' 'c4b SVS_POA_QUEUE_ORDER=2' 'c8b SVS_POA_QUEUE_ORDER=3' 'c2b SVS_POA_QUEUE_ORDER=4'
