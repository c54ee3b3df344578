set -o pipefail
# Two more samples of the driver's command on the final tree (r02_v43's run
# had the host fold 20 % slower than r02_v38's box: host-side spread).
D=gpurun_out/r02_v45
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-sample 0 > $D/bench_driver_cmd_1.log 2>&1 && \
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-sample 0 > $D/bench_driver_cmd_2.log 2>&1
