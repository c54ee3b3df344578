set -o pipefail
D=gpurun_out/r03_v26
mkdir -p $D
export TMPDIR=/tmp
SVS_LIB_PATH=$PWD/svscope_amd/lib/variants/libsvscope_hip_foldexam.so SVS_POA_FOLD_TIMES=1 timeout -k 10 300 python -u tools/poa_probe.py --windows 8 > $D/probe8.json 2> $D/probe8.err || { tail -30 $D/probe8.err; exit 1; }
grep "svs\]" $D/probe8.err
