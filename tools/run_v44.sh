set -o pipefail
mkdir -p gpurun_out/v44
export TMPDIR=/tmp
for a in 768 1280; do
  timeout -k 10 300 env SVS_POA_ACTIVE_JOBS=$a python -u bench.py --cpu-sample 0 > gpurun_out/v44/bench_active_$a.log 2>&1 || exit 1
done
