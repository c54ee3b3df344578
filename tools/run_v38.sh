set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/prof_v38
mkdir -p $OUT
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/bench_ktrace -o run -- python3 bench.py --cpu-sample 0 > $OUT/bench_under_rocprof.log 2>&1 && \
python3 tools/prof_summary.py stats $OUT/bench_ktrace > $OUT/bench_ktrace_stats.json && \
timeout -k 10 900 bash tools/profile_poa.sh v38 512
