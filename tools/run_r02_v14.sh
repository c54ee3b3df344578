set -o pipefail
D=gpurun_out/r02_v14
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_poa_gpu.py -x -v --timeout 120 --timeout-method thread -k "variants" > $D/pytest_variants.log 2>&1 && \
timeout -k 10 200 python -u tools/poa_probe.py --windows 2048 > $D/probe_narrow.log 2>&1 && \
SVS_POA_WIDE=1 timeout -k 10 200 python -u tools/poa_probe.py --windows 2048 --check 2 > $D/probe_wide.log 2>&1 && \
SVS_POA_WIDE=1 timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench_wide.log 2>&1
