set -o pipefail
mkdir -p gpurun_out/v43
export TMPDIR=/tmp
for s in 0.02 0.03 0.08; do
  timeout -k 10 300 env SVS_POA_PRUNE_SLACK=$s python -u bench.py --cpu-sample 0 > gpurun_out/v43/bench_slack_$s.log 2>&1 || exit 1
done
