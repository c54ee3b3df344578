set -o pipefail
# Export kernel: previous-chunk register windows + lazily drained scratch
# (product lib) vs HEAD (variants/..._head.so) on the MSA probe, then the
# round's evidence pass on the product lib: GPU suite, smoke, driver bench,
# rocprofv3 kernel stats, PMC HBM traffic.
D=gpurun_out/r02_v33
mkdir -p $D
export TMPDIR=/tmp
HEADLIB=$PWD/svscope_amd/lib/variants/libsvscope_hip_head.so
p() { timeout -k 10 200 python -u tools/poa_probe.py --windows 2048 > $D/probe_$1.log 2>&1; }
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $D/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 && \
SVS_LIB_PATH=$HEADLIB p head1 && p new1 && SVS_LIB_PATH=$HEADLIB p head2 && p new2 && \
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench_driver_cmd.log 2>&1 && \
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $D/bench_ktrace -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-sample 0 > $D/bench_under_rocprof.log 2>&1 && \
bash tools/profile_bench_pmc.sh r02_v33/pmc > $D/pmc_poa_traffic.json 2> $D/pmc.err
