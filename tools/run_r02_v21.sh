set -o pipefail
D=gpurun_out/r02_v21
mkdir -p $D
export TMPDIR=/tmp
p() { timeout -k 10 200 python -u tools/poa_probe.py --windows 2048 > $D/probe_$1.log 2>&1; }
b() { timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-sample 0 > $D/bench_$1.log 2>&1; }
SVS_POA_JOB_ORDER=0 p off1 && p on1 && SVS_POA_JOB_ORDER=0 p off2 && p on2 && \
SVS_POA_JOB_ORDER=0 b off1 && b on1 && SVS_POA_JOB_ORDER=0 b off2 && b on2
