set -o pipefail
mkdir -p gpurun_out/v41
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_misscore_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/v41/pytest_misscore.log 2>&1 && \
timeout -k 10 300 python -u tools/misscore_probe.py --pairs 4096 > gpurun_out/v41/ms_probe.log 2>&1 && \
timeout -k 10 300 env SVS_MS_FILL=32 python -u tools/misscore_probe.py --pairs 4096 --cpu-sample 0 > gpurun_out/v41/ms_probe_int32.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/v41/ms_ktrace -o run -- python3 tools/misscore_probe.py --pairs 4096 --reps 1 --cpu-sample 0 > gpurun_out/v41/ms_prof.log 2>&1
