set -o pipefail
mkdir -p gpurun_out/v49
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_decision_gpu.py -x -v --timeout 240 --timeout-method thread > gpurun_out/v49/pytest_decision.log 2>&1 && \
for p in 1.5 1.0 -1; do
  timeout -k 10 400 env SVS_POA_CONS_PRIOR=$p python -u bench.py --cpu-sample 0 > gpurun_out/v49/bench_prior_$p.log 2>&1 || exit 1
done
