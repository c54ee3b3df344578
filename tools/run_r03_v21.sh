set -o pipefail
D=gpurun_out/r03_v21
mkdir -p $D
export TMPDIR=/tmp
SVS_LIB_PATH=$PWD/svscope_amd/lib/variants/libsvscope_hip_foldprof.so SVS_POA_FOLD_TIMES=1 timeout -k 10 300 python -u tools/poa_probe.py --windows 8 > $D/probe8.json 2> $D/probe8.err || { tail -30 $D/probe8.err; exit 1; }
grep "svs\]" $D/probe8.err
SVS_LIB_PATH=$PWD/svscope_amd/lib/variants/libsvscope_hip_foldprof.so SVS_POA_FOLD_TIMES=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-sample 0 > $D/bench.json 2> $D/bench.err || { tail -30 $D/bench.err; exit 1; }
grep "svs\]" $D/bench.err
