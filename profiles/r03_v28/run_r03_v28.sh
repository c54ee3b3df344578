set -o pipefail
D=gpurun_out/r03_v28
mkdir -p $D
export TMPDIR=/tmp
V=$PWD/svscope_amd/lib/variants/libsvscope_hip_occ7.so
SVS_LIB_PATH=$V timeout -k 10 200 python -u -m pytest tests/test_poa_gpu.py -x -q --timeout 120 --timeout-method thread -k "random_cases_batched or kernel_variants or wide_traceback" > $D/t0.log 2>&1 || { tail -30 $D/t0.log; exit 1; }
tail -2 $D/t0.log
run() { n=$1; shift; env "$@" timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --cpu-sample 0 > $D/b_$n.json 2> $D/b_$n.err; }
run base SVS_X=0 && run occ7 SVS_LIB_PATH=$V && run base2 SVS_X=0 && run occ7b SVS_LIB_PATH=$V
rc=$?
for f in $D/b_*.json; do python3 -c "import json,sys; d=json.load(open('$f')); print('$f', d['value'], d['roofline']['mean_launch_ms'], d['breakdown']['poa_launches'], d['oracle_check']['match'])"; done
exit $rc
