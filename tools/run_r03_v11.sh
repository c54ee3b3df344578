set -o pipefail
D=gpurun_out/r03_v11
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --cpu-sample 0 > $D/b_default.json 2> $D/b_default.err && \
SVS_POA_STREAMS=2 timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --cpu-sample 0 > $D/b_streams2.json 2> $D/b_streams2.err && \
SVS_POA_STREAMS=2 SVS_POA_ACTIVE_JOBS=768 timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --cpu-sample 0 > $D/b_streams2_aj768.json 2> $D/b_streams2_aj768.err
rc=$?
for f in $D/b_*.json; do python3 -c "import json,sys; d=json.load(open('$f')); print('$f', d['value'], d['roofline']['mean_launch_ms'], d['breakdown']['poa_launches'])"; done
exit $rc
