set -o pipefail
mkdir -p gpurun_out/r06_m1
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_a_multirank_gpu.py -x -v -s --timeout 400 --timeout-method thread > gpurun_out/r06_m1/pytest.log 2>&1 || { tail -40 gpurun_out/r06_m1/pytest.log; exit 1; }
tail -3 gpurun_out/r06_m1/pytest.log
grep '^{' gpurun_out/r06_m1/pytest.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ranks'], d['oracle_check']['match'])"
SVS_DEVICE=0 SVS_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --steps 4 --warmup 1 --cpu-sample 0 > gpurun_out/r06_m1/bench2.log 2>&1 || { tail -30 gpurun_out/r06_m1/bench2.log; exit 1; }
tail -1 gpurun_out/r06_m1/bench2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], json.dumps(d['ranks']), d['oracle_check']['windows_checked'] if 'windows_checked' in d['oracle_check'] else d['oracle_check'])"
