#!/bin/bash
# Evidence pass on the GPU box: the GPU test suite, smoke(), the driver's bench
# command, and the same bench under a rocprofv3 kernel trace (+ the HIP-event
# vs rocprofv3 comparison).  Optional PMC / SQ passes with EXTRA=1.
#   tools/evidence_pass.sh NAME        (writes gpurun_out/NAME/)
set -o pipefail
N=${1:?name}
D=gpurun_out/$N
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { tail -30 $D/pytest_gpu.log; exit 1; }
tail -2 $D/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench_driver_cmd.log 2>&1 || { tail -20 $D/bench_driver_cmd.log; exit 1; }
tail -1 $D/bench_driver_cmd.log
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $D/bench_ktrace -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-sample 0 > $D/bench_under_rocprof.log 2>&1 || { tail -20 $D/bench_under_rocprof.log; exit 1; }
python3 tools/rocprof_timed.py $D/bench_ktrace $D/bench_under_rocprof.log > $D/bench_under_rocprof.json || exit 1
cp $(find $D/bench_ktrace -name '*kernel_stats.csv' | head -1) $D/bench_kernel_stats.csv
if [ -n "$EXTRA" ]; then
  bash tools/profile_bench_pmc.sh $N/pmc > $D/pmc_poa_traffic.json 2> $D/pmc.err || exit 1
  bash tools/profile_bench_sq.sh $N/sq > $D/sq_poa_bench.json 2> $D/sq.err || exit 1
fi
echo done
