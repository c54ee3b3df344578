#!/bin/bash
# rocprofv3 evidence for the POA kernel (run on the GPU box from the repo root):
#   kernel trace + stats, then FETCH_SIZE, WRITE_SIZE and SQ counter passes,
#   each its own rocprofv3 run (no --pmc together with sys/runtime traces).
# usage: tools/profile_poa.sh TAG WINDOWS
set -e
TAG=${1:-r01}; W=${2:-512}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name, rocprofv3 args...
  local name=$1; shift
  timeout -k 10 400 rocprofv3 "$@" --output-format csv -d $OUT/$name -o run -- python3 tools/poa_probe.py --windows $W > $OUT/$name.log 2>&1
}
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
have() {  # keep only counters this agent lists
  local keep=""
  for c in "$@"; do grep -qw "$c" $OUT/counters.txt && keep="$keep $c"; done
  echo $keep
}
run ktrace --kernel-trace --stats
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
SQ1=$(have SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU)
SQ2=$(have SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH)
echo "sq1: $SQ1" > $OUT/sq_counters.txt; echo "sq2: $SQ2" >> $OUT/sq_counters.txt
run sq1 --pmc $SQ1
# SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
run sq2 --pmc $SQ2
python3 tools/prof_summary.py stats $OUT/ktrace > $OUT/ktrace_stats.json
for p in fetch write sq1 sq2; do python3 tools/prof_summary.py pmc $OUT/$p $OUT/$p.log > $OUT/$p.json; done
python3 tools/prof_summary.py merge $OUT/pmc_poa_traffic.json $OUT/fetch.json $OUT/write.json
