set -o pipefail
D=gpurun_out/r03_v10
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $D/kdev -o run -- python3 bench.py --gpus 1 --steps 6 --warmup 1 --cpu-sample 0 > $D/bench_dev.log 2>&1 && \
SVS_POA_HOST_GRAPH=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $D/khost -o run -- python3 bench.py --gpus 1 --steps 6 --warmup 1 --cpu-sample 0 > $D/bench_host.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d $D/sq1 -o run -- python3 bench.py --steps 2 --warmup 0 --cpu-sample 0 > $D/sq1.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH --output-format csv -d $D/sq2 -o run -- python3 bench.py --steps 2 --warmup 0 --cpu-sample 0 > $D/sq2.log 2>&1
rc=$?
for k in kdev khost; do python3 tools/ktrace_overlap.py $D/$k > $D/$k.json 2>&1; done
exit $rc
