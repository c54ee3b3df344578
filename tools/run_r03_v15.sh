set -o pipefail
D=gpurun_out/r03_v15
mkdir -p $D
export TMPDIR=/tmp
SVS_POA_VERIFY_GRAPH=1 timeout -k 10 120 python -u -m pytest tests/test_poa_gpu.py -x -v --timeout 100 --timeout-method thread -k "random_cases_batched or handchecked or device_graphs" > $D/t0.log 2>&1 || { tail -30 $D/t0.log; exit 1; }
tail -2 $D/t0.log
timeout -k 10 300 python -u -m pytest tests/test_poa_gpu.py tests/test_decision_gpu.py -x -v --timeout 120 --timeout-method thread > $D/t1.log 2>&1 || { tail -40 $D/t1.log; exit 1; }
tail -2 $D/t1.log
SVS_POA_FOLD_TIMES=1 timeout -k 10 300 python -u bench.py --cpu-sample 0 > $D/bench.json 2> $D/bench.err || { tail -30 $D/bench.err; exit 1; }
grep "fold times" $D/bench.err
python3 -c "import json; d=json.load(open('$D/bench.json')); print(d['value'], d['roofline']['mean_launch_ms'], d['breakdown']['poa_launches'], d['oracle_check']['match'])"
