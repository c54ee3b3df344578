set -o pipefail
D=gpurun_out/r03_v4
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $D/ktrace -o run -- python3 bench.py --gpus 1 --steps 6 --warmup 1 --cpu-sample 0 > $D/bench.log 2>&1
