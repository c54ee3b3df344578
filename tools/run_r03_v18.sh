set -o pipefail
D=gpurun_out/r03_v18
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $D/kdev -o run -- python3 bench.py --gpus 1 --steps 6 --warmup 1 --cpu-sample 0 > $D/bench_dev.log 2>&1
rc=$?
python3 tools/gap_report.py $D/kdev 12
python3 tools/ktrace_overlap.py $D/kdev > $D/kdev.json
exit $rc
