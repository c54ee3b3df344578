set -o pipefail
D=gpurun_out/r03_v16
mkdir -p $D
export TMPDIR=/tmp
SVS_POA_FOLD_TIMES=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-sample 0 > $D/bench.json 2> $D/bench.err || { tail -30 $D/bench.err; exit 1; }
grep "fold times" $D/bench.err
SVS_POA_FOLD_TIMES=1 timeout -k 10 300 python -u tools/poa_probe.py --windows 8 > $D/probe8.json 2> $D/probe8.err || { tail -30 $D/probe8.err; exit 1; }
grep "fold times" $D/probe8.err
