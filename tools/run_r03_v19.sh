set -o pipefail
D=gpurun_out/r03_v19
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_poa_gpu.py -x -v --timeout 150 --timeout-method thread -k "many_in_edges" > $D/t0.log 2>&1; rc0=$?
tail -5 $D/t0.log
timeout -k 10 300 python -u -m pytest tests/test_decision_gpu.py -x -v --timeout 250 --timeout-method thread -k "big_windows" > $D/t1.log 2>&1; rc1=$?
tail -15 $D/t1.log
[ $rc0 -eq 0 ] && [ $rc1 -eq 0 ] || exit 1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $D/t2.log 2>&1 || { tail -30 $D/t2.log; exit 1; }
tail -2 $D/t2.log
