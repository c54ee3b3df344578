set -o pipefail
D=gpurun_out/r02_v11
mkdir -p $D
export TMPDIR=/tmp
for v in base nodm all3; do
  if [ $v = base ]; then unset SVS_LIB_PATH; else export SVS_LIB_PATH=$PWD/svscope_amd/lib/variants/libsvscope_hip_$v.so; fi
  timeout -k 10 200 python -u tools/poa_probe.py --windows 2048 > $D/probe_$v.log 2>&1 || exit 1
done
unset SVS_LIB_PATH
SVS_POA_TRACE=$D/trace_b512.txt timeout -k 10 300 python -u bench.py --steps 6 --warmup 1 --cpu-sample 0 > $D/bench_trace.log 2>&1
