set -o pipefail
mkdir -p gpurun_out/v48
export TMPDIR=/tmp
for i in 1 2; do
  for b in 2048 4096; do
    timeout -k 10 400 python -u bench.py --cpu-sample 0 --batch $b > gpurun_out/v48/bench_b${b}_$i.log 2>&1 || exit 1
  done
done
