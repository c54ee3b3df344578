set -o pipefail
D=gpurun_out/r03_v7
mkdir -p $D
export TMPDIR=/tmp
SVS_POA_DEBUG=1 SVS_POA_SYNC_CHECK=1 timeout -k 10 60 python -u -m pytest tests/test_poa_gpu.py -x -v -s --timeout 45 --timeout-method thread -k "random_cases_batched" > $D/t2.log 2>&1 || { grep "svs\]" $D/t2.log | tail -30; exit 1; }
tail -3 $D/t2.log
