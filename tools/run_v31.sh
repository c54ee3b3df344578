set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/v31
mkdir -p $OUT
SQ1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
SQ2="SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH"
for v in prune noprune; do
  if [ $v = noprune ]; then export SVS_POA_PRUNE=0; else unset SVS_POA_PRUNE; fi
  timeout -s KILL 300 rocprofv3 --pmc $SQ1 --output-format csv -d $OUT/${v}_sq1 -o run -- python3 tools/poa_probe.py --windows 512 > $OUT/${v}_sq1.log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc $SQ2 --output-format csv -d $OUT/${v}_sq2 -o run -- python3 tools/poa_probe.py --windows 512 > $OUT/${v}_sq2.log 2>&1
  python3 tools/prof_summary.py pmc $OUT/${v}_sq1 $OUT/${v}_sq1.log > $OUT/${v}_sq1.json
  python3 tools/prof_summary.py pmc $OUT/${v}_sq2 $OUT/${v}_sq2.log > $OUT/${v}_sq2.json
done
