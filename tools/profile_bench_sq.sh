#!/bin/bash
# SQ counters of every kernel on the bench workload (one 512-window step, no
# warm-up), two passes of at most 8 SQ counters each; per-strip-row figures for
# the POA strip kernel, per-kernel sums for all of them (the fold kernels share
# the CUs with it).
set -e
OUT=gpurun_out/${1:-prof_bench_sq}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d $OUT/sq1 -o run -- python3 bench.py --steps 1 --warmup 0 --cpu-sample 0 > $OUT/sq1.log 2>&1
timeout -s KILL 600 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH --output-format csv -d $OUT/sq2 -o run -- python3 bench.py --steps 1 --warmup 0 --cpu-sample 0 > $OUT/sq2.log 2>&1
python3 - "$OUT" <<'PY'
import collections, csv, glob, json, re, sys
out = sys.argv[1]
res = {}
per_kernel = collections.defaultdict(lambda: collections.defaultdict(float))
cells = None
for p in ("sq1", "sq2"):
    for f in glob.glob(f"{out}/{p}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            name = re.sub(r"\(.*", "", row["Kernel_Name"]).replace("void ", "")
            per_kernel[name][row["Counter_Name"]] += float(row["Counter_Value"])
            if "poa_strip_kernel" in row["Kernel_Name"]:
                res[row["Counter_Name"]] = res.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    line = [l for l in open(f"{out}/{p}.log") if l.startswith("{")][-1]
    cells = json.loads(line)["breakdown"]["poa_cells_computed"]
strip_rows = cells / 64
per_row = {k: v / strip_rows for k, v in res.items() if k.startswith("SQ_INSTS")}
if res.get("SQ_WAVE_CYCLES"):
    per_row["wait_any_over_wave_cycles"] = res.get("SQ_WAIT_ANY", 0.0) / res["SQ_WAVE_CYCLES"]
print(json.dumps({"kernel": "poa_strip_kernel", "workload": "bench.py --steps 1 --warmup 0 (one 512-window config-3 step)",
                  "cells_computed": cells, "counter_sums": res, "per_strip_row": per_row,
                  "per_kernel": {k: dict(v) for k, v in per_kernel.items()}}, indent=1))
PY
