set -o pipefail
D=gpurun_out/r03_v27
mkdir -p $D
export TMPDIR=/tmp
SVS_POA_VERIFY_GRAPH=1 timeout -k 10 150 python -u -m pytest tests/test_poa_gpu.py -x -v --timeout 120 --timeout-method thread -k "random_cases_batched or handchecked or device_graphs or wide_traceback" > $D/t0.log 2>&1 || { tail -30 $D/t0.log; exit 1; }
tail -2 $D/t0.log
SVS_LIB_PATH=$PWD/svscope_amd/lib/variants/libsvscope_hip_foldexam.so SVS_POA_FOLD_TIMES=1 timeout -k 10 300 python -u tools/poa_probe.py --windows 8 > $D/probe8x.json 2> $D/probe8x.err || { tail -30 $D/probe8x.err; exit 1; }
grep "svs\]" $D/probe8x.err
SVS_POA_FOLD_TIMES=1 timeout -k 10 300 python -u tools/poa_probe.py --windows 8 > $D/probe8.json 2> $D/probe8.err || { tail -30 $D/probe8.err; exit 1; }
grep "svs\]" $D/probe8.err
