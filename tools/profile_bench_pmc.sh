#!/bin/bash
# PMC HBM traffic of the POA strip kernel on the bench workload itself:
# FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes over one timed bench
# step (no warm-up, so every strip dispatch is inside the step whose
# cells_computed the bench reports), summed over strip-kernel dispatches.
set -e
OUT=gpurun_out/${1:-prof_bench_pmc}
mkdir -p $OUT
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 600 rocprofv3 --pmc $c --output-format csv -d $OUT/$c -o run -- python3 bench.py --steps 1 --warmup 0 --cpu-sample 0 > $OUT/$c.log 2>&1
done
python3 - "$OUT" <<'PY'
import csv, glob, json, sys
out = sys.argv[1]
tot = {}
n = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob(f"{out}/{c}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if "poa_strip_kernel" in row["Kernel_Name"]:
                tot[c] = tot.get(c, 0.0) + float(row["Counter_Value"])
                n[c] = n.get(c, 0) + 1
res = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    line = [l for l in open(f"{out}/{c}.log") if l.startswith("{")][-1]
    b = json.loads(line)["breakdown"]
    res[c] = {"kB": tot.get(c, 0.0), "dispatches": n.get(c, 0), "cells_computed": b["poa_cells_computed"],
              "launches": b["poa_launches"]}
fb = res["FETCH_SIZE"]["kB"] * 1024 * 2
wb = res["WRITE_SIZE"]["kB"] * 1024
cf, cw = res["FETCH_SIZE"]["cells_computed"], res["WRITE_SIZE"]["cells_computed"]
print(json.dumps({"kernel": "poa_strip_kernel",
                  "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over bench.py --steps 1 --warmup 0; kB x 1024; FETCH_SIZE doubled (gfx950 under-count, MI355X_MICROARCH.md HBM section)",
                  "fetch_bytes_per_cell": fb / cf, "fetch_bytes_per_cell_raw": fb / 2 / cf,
                  "write_bytes_per_cell": wb / cw, "hbm_bytes_per_cell": fb / cf + wb / cw,
                  "per": "DP cell evaluated by the kernel (cells_computed)", "passes": res}, indent=1))
PY
