#!/bin/bash
# Bench evidence on the GPU box: smoke(), the driver's bench command, the same
# bench under a rocprofv3 kernel trace (HIP-event vs rocprofv3 DP means; the
# timed span's per-kernel totals and overlap), then the counters of the timed
# DP instance (tools/profile_instance.sh).  Writes gpurun_out/NAME/.
#   tools/evidence_bench.sh NAME [skip_counters]
set -o pipefail
N=${1:?name}
D=gpurun_out/$N
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench_driver_cmd.log 2>&1 || { tail -20 $D/bench_driver_cmd.log; exit 1; }
tail -1 $D/bench_driver_cmd.log | cut -c1-400
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $D/bench_ktrace -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-sample 0 > $D/bench_under_rocprof.log 2>&1 || { tail -20 $D/bench_under_rocprof.log; exit 1; }
python3 tools/rocprof_timed.py $D/bench_ktrace $D/bench_under_rocprof.log > $D/bench_under_rocprof.json || exit 1
python3 tools/ktrace_overlap.py $D/bench_ktrace > $D/ktrace_overlap.json || exit 1
cp $(find $D/bench_ktrace -name '*kernel_stats.csv' | head -1) $D/bench_kernel_stats.csv
rm -rf $D/bench_ktrace
[ -n "$2" ] && { echo done; exit 0; }
bash tools/profile_instance.sh $N/counters 4 > $D/profile_instance.log 2>&1 || { tail -20 $D/profile_instance.log; exit 1; }
tail -1 $D/profile_instance.log
echo done
