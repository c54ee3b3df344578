set -o pipefail
D=gpurun_out/r03_v22
mkdir -p $D
export TMPDIR=/tmp
rm -f $D/trace.txt
SVS_POA_TRACE=$D/trace.txt timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --cpu-sample 0 > $D/bench.json 2> $D/bench.err || { tail -30 $D/bench.err; exit 1; }
python3 tools/poa_timeline.py $D/trace.txt > $D/timeline.txt
tail -20 $D/timeline.txt
