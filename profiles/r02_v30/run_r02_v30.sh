set -o pipefail
# A/B: DPP scans as builtins + branch-free in-edge liveness (new, product lib)
# against the previous commit's library (variants/libsvscope_hip_old.so)
D=gpurun_out/r02_v30
mkdir -p $D
export TMPDIR=/tmp
OLD=$PWD/svscope_amd/lib/variants/libsvscope_hip_old.so
p() { timeout -k 10 200 python -u tools/poa_probe.py --windows 2048 > $D/probe_$1.log 2>&1; }
timeout -k 10 400 python -u -m pytest tests/test_poa_gpu.py tests/test_decision_gpu.py -x -v --timeout 240 --timeout-method thread > $D/pytest_poa.log 2>&1 && \
SVS_LIB_PATH=$OLD p old1 && p new1 && SVS_LIB_PATH=$OLD p old2 && p new2 && \
bash tools/profile_bench_sq.sh r02_v30/sq_new > $D/sq_new.json 2> $D/sq_new.err && \
SVS_LIB_PATH=$OLD bash tools/profile_bench_sq.sh r02_v30/sq_old > $D/sq_old.json 2> $D/sq_old.err
