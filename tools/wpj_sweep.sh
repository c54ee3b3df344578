#!/bin/bash
# Waves-per-job sweep of the strip kernel on the MSA probe (GPU box).
# usage: tools/wpj_sweep.sh WINDOWS "4 6 8" OUTDIR
W=${1:-2048}; LIST=${2:-"4 6 8"}; OUT=${3:-gpurun_out/wpj_sweep}
mkdir -p $OUT
for w in $LIST; do
  SVS_POA_WPJ=$w timeout -k 10 300 python tools/poa_probe.py --windows $W > $OUT/w${W}_wpj$w.log 2>&1 || exit 1
  echo "wpj=$w $(grep gcups_kernel $OUT/w${W}_wpj$w.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["gcups_kernel"],1), "GCUPS", round(d["windows_per_s"],1), "win/s")')"
done
SVS_POA_WPJ_RESIDENT=1 SVS_POA_DEBUG=1 timeout -k 10 300 python tools/poa_probe.py --windows $W > $OUT/w${W}_resident.log 2>&1 || exit 1
echo "resident: $(grep -m3 'strip launch' $OUT/w${W}_resident.log | tail -1) $(grep gcups_kernel $OUT/w${W}_resident.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["gcups_kernel"],1), "GCUPS")')"
