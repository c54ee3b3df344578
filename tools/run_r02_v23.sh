set -o pipefail
D=gpurun_out/r02_v23
mkdir -p $D
export TMPDIR=/tmp
p() { timeout -k 10 200 python -u tools/poa_probe.py --windows 2048 > $D/probe_$1.log 2>&1; }
b() { timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-sample 0 > $D/bench_$1.log 2>&1; }
p base && SVS_POA_STREAMS=2 p s2 && p base2 && SVS_POA_STREAMS=2 p s2b && \
b base && SVS_POA_STREAMS=2 b s2 && b base2 && SVS_POA_STREAMS=2 b s2b
