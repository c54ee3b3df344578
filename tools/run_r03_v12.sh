set -o pipefail
D=gpurun_out/r03_v12
mkdir -p $D
export TMPDIR=/tmp
run() { n=$1; shift; env "$@" timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --cpu-sample 0 > $D/b_$n.json 2> $D/b_$n.err; }
run default SVS_X=0 && run aj1536 SVS_POA_ACTIVE_JOBS=1536 && run aj2048 SVS_POA_ACTIVE_JOBS=2048 && run s2aj1536 SVS_POA_STREAMS=2 SVS_POA_ACTIVE_JOBS=1536 && run default2 SVS_X=0
rc=$?
for f in $D/b_*.json; do python3 -c "import json,sys; d=json.load(open('$f')); print('$f', d['value'], d['roofline']['mean_launch_ms'], d['breakdown']['poa_launches'], d['breakdown']['poa_kernel_ms'])"; done
exit $rc
SVS_POA_FOLD_TIMES=1 timeout -k 10 200 python3 bench.py --steps 4 --warmup 1 --cpu-sample 0 > $D/b_ft.json 2> $D/b_ft.err
grep "fold times" $D/b_ft.err
