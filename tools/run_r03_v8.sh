set -o pipefail
D=gpurun_out/r03_v8
mkdir -p $D
export TMPDIR=/tmp
SVS_POA_DEBUG=1 SVS_POA_SYNC_CHECK=1 SVS_POA_VERIFY_GRAPH=1 timeout -k 10 90 python -u -m pytest tests/test_poa_gpu.py -x -v -s --timeout 60 --timeout-method thread -k "random_cases_batched or handchecked" > $D/t1.log 2>&1 || { grep "svs\]" $D/t1.log | tail -30; tail -30 $D/t1.log; exit 1; }
tail -3 $D/t1.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $D/t2.log 2>&1 || { tail -40 $D/t2.log; exit 1; }
tail -3 $D/t2.log
timeout -k 10 300 python -u bench.py > $D/bench.json 2> $D/bench.err || { tail -30 $D/bench.err; exit 1; }
cat $D/bench.json
