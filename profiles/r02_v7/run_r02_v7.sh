set -o pipefail
D=gpurun_out/r02_v7
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $D/rocprof_counters.txt 2>&1 || true
timeout -k 10 300 python -u tools/prune_probe.py --windows 512 --error 0.08 --ins-min 200 --ins-max 801 --check 1 > $D/prune_default.log 2>&1 && \
timeout -k 10 400 python -u tools/prune_probe.py --windows 512 --check 2 > $D/prune_harsh.log 2>&1 && \
SVS_POA_PRUNE_SLACK=0.08 timeout -k 10 300 python -u tools/prune_probe.py --windows 512 > $D/prune_harsh_slack08.log 2>&1 && \
SVS_POA_PRUNE_SLACK=0.12 timeout -k 10 300 python -u tools/prune_probe.py --windows 512 > $D/prune_harsh_slack12.log 2>&1 && \
SVS_POA_PRUNE=0 timeout -k 10 400 python -u tools/prune_probe.py --windows 512 > $D/prune_harsh_off.log 2>&1
