set -o pipefail
mkdir -p gpurun_out/v57
export TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 400 python -u bench.py --cpu-sample 0 > gpurun_out/v57/bench_$i.log 2>&1 || exit 1
done
