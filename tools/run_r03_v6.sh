set -o pipefail
D=gpurun_out/r03_v6
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_poa_gpu.py -x -v --timeout 300 --timeout-method thread -k "device_graphs or random_cases_batched or variants" > $D/t.log 2>&1 && \
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $D/ktrace -o run -- python3 bench.py --gpus 1 --steps 6 --warmup 1 --cpu-sample 0 > $D/bench.log 2>&1
rc=$?; tail -3 $D/t.log; exit $rc
