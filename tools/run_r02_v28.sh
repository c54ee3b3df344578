set -o pipefail
D=gpurun_out/r02_v28
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_poa_gpu.py -x -v --timeout 180 --timeout-method thread > $D/pytest_poa.log 2>&1 || exit 1
p() { timeout -k 10 200 python -u tools/poa_probe.py --windows 2048 > $D/probe_$1.log 2>&1; }
b() { timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-sample 0 > $D/bench_$1.log 2>&1; }
SVS_POA_DEVICE_PREP=0 p host && p dev && SVS_POA_PREP_STREAM=1 p devs && \
SVS_POA_DEVICE_PREP=0 b host && b dev && SVS_POA_PREP_STREAM=1 b devs && SVS_POA_DEVICE_PREP=0 b host2 && b dev2 && SVS_POA_PREP_STREAM=1 b devs2
