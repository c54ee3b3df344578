set -o pipefail
D=gpurun_out/r03_v24
mkdir -p $D
export TMPDIR=/tmp
SVS_POA_FOLD_CUS=32 SVS_POA_VERIFY_GRAPH=1 timeout -k 10 150 python -u -m pytest tests/test_poa_gpu.py -x -v --timeout 120 --timeout-method thread -k "random_cases_batched or device_graphs" > $D/t0.log 2>&1 || { tail -30 $D/t0.log; exit 1; }
tail -2 $D/t0.log
run() { n=$1; shift; env "$@" timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --cpu-sample 0 > $D/b_$n.json 2> $D/b_$n.err; }
run cu0 SVS_POA_FOLD_CUS=0 && run cu32 SVS_POA_FOLD_CUS=32 && run cu16 SVS_POA_FOLD_CUS=16 && run cu64 SVS_POA_FOLD_CUS=64 && run cu0b SVS_POA_FOLD_CUS=0
rc=$?
for f in $D/b_*.json; do python3 -c "import json,sys; d=json.load(open('$f')); print('$f', d['value'], d['roofline']['mean_launch_ms'], d['breakdown']['poa_launches'], d['oracle_check'])"; done
exit $rc
