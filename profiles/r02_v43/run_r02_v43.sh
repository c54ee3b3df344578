set -o pipefail
# Evidence pass on the final round-2 tree:
D=gpurun_out/r02_v43
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $D/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 && \
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench_driver_cmd.log 2>&1 && \
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $D/bench_ktrace -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-sample 0 > $D/bench_under_rocprof.log 2>&1 && \
bash tools/profile_bench_pmc.sh r02_v43/pmc > $D/pmc_poa_traffic.json 2> $D/pmc.err && \
bash tools/profile_bench_sq.sh r02_v43/sq > $D/sq_poa_bench.json 2> $D/sq.err
