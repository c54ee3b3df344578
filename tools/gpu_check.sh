#!/bin/bash
# GPU-box check: the GPU test suite, then a short bench line.
#   tools/gpu_check.sh OUT_DIR [BENCH_STEPS]
OUT=${1:-gpurun_out/check}; STEPS=${2:-4}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 400 python bench.py --steps $STEPS --warmup 1 --cpu-sample 0 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
