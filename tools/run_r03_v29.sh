set -o pipefail
D=gpurun_out/r03_v29
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_decision_gpu.py -x -v --timeout 250 --timeout-method thread -k "engine_limit or big_windows" > $D/t0.log 2>&1 || { tail -40 $D/t0.log; exit 1; }
tail -3 $D/t0.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 250 --timeout-method thread > $D/t1.log 2>&1 || { tail -30 $D/t1.log; exit 1; }
tail -2 $D/t1.log
timeout -k 10 300 python -u bench.py > $D/bench.json 2> $D/bench.err || { tail -30 $D/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$D/bench.json')); print(d['value'], d['roofline']['mean_launch_ms'], d['breakdown']['poa_launches'], d['oracle_check']['match'], d['breakdown']['host_graph_ms'])"
