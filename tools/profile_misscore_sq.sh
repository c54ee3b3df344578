#!/bin/bash
# SQ counters of the MisScore kernels over one probe call (4096 pairs).
set -e
OUT=gpurun_out/${1:-prof_ms_sq}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/sq -o run -- python3 tools/misscore_probe.py --pairs 4096 --reps 1 --cpu-sample 0 --check 0 --warmup 0 > $OUT/sq.log 2>&1
python3 - "$OUT" <<'PY'
import csv, glob, json, re, sys
out = sys.argv[1]
res = {}
for f in glob.glob(f"{out}/sq/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        m = re.search(r"(\w+_kernel)", row["Kernel_Name"])
        k = m.group(1) if m else "other"
        d = res.setdefault(k, {})
        d[row["Counter_Name"]] = d.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
probe = [json.loads(l) for l in open(f"{out}/sq.log") if l.startswith("{")]
print(json.dumps({"counters": res, "probe": probe[-1] if probe else None}, indent=1))
PY
