set -o pipefail
# A/B: DPP scans as builtins, 32-bit record/carry offsets, prep scratch in LDS
# (product lib) against the round's previous commit (variants/..._old.so)
D=gpurun_out/r02_v31
mkdir -p $D
export TMPDIR=/tmp
OLD=$PWD/svscope_amd/lib/variants/libsvscope_hip_old.so
p() { timeout -k 10 200 python -u tools/poa_probe.py --windows 2048 > $D/probe_$1.log 2>&1; }
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $D/pytest_gpu.log 2>&1 && \
SVS_LIB_PATH=$OLD p old1 && p new1 && SVS_LIB_PATH=$OLD p old2 && p new2 && \
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench_new.log 2>&1 && \
SVS_LIB_PATH=$OLD timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-sample 0 > $D/bench_old.log 2>&1
