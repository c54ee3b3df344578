set -o pipefail
# Export kernel: chain rows (one in-edge from the row above; no slot for the
# slot pass) skipped by the sequential slot and source-distance passes and
# short-cut in the sink-distance pass; tables verified before the DP kernel
# (SVS_POA_VERIFY_PREP). A/B on the MSA probe against the r02_v38 library;
# latefetch = + the strip kernel's record/carry prefetch issued mid-row, after
# the row's pool reads (SVS_LATE_FETCH). Then a traced bench run.
D=gpurun_out/r02_v39
mkdir -p $D
export TMPDIR=/tmp
V=$PWD/svscope_amd/lib/variants
p() { timeout -k 10 200 python -u tools/poa_probe.py --windows 2048 > $D/probe_$1.log 2>&1; }
timeout -k 10 400 python -u -m pytest tests/test_poa_gpu.py tests/test_decision_gpu.py -x -v --timeout 240 --timeout-method thread > $D/pytest_poa.log 2>&1 && \
SVS_LIB_PATH=$V/libsvscope_hip_latefetch.so timeout -k 10 400 python -u -m pytest tests/test_poa_gpu.py -x -v --timeout 240 --timeout-method thread -k "variants or oracle or config3" > $D/pytest_latefetch.log 2>&1 && \
SVS_LIB_PATH=$V/libsvscope_hip_v38.so p v38a && p new1 && SVS_LIB_PATH=$V/libsvscope_hip_latefetch.so p lf1 && \
SVS_LIB_PATH=$V/libsvscope_hip_v38.so p v38b && p new2 && SVS_LIB_PATH=$V/libsvscope_hip_latefetch.so p lf2 && \
SVS_POA_TRACE=$D/trace_b512.txt timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --cpu-sample 0 > $D/bench_trace.log 2>&1
