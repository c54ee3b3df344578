set -o pipefail
D=gpurun_out/r02_v20
mkdir -p $D
export TMPDIR=/tmp
b() { timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-sample 0 "${@:2}" > $D/bench_$1.log 2>&1; }
b d4a --depth 4 && b d6a --depth 6 && b d5a --depth 5 && b d6b --depth 6 && b d4b --depth 4 && b d7a --depth 7
