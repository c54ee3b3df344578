#!/bin/bash
# rocprofv3 PMC evidence for the MisScore kernels (run on the GPU box from the
# repo root): FETCH_SIZE and WRITE_SIZE in separate passes over one probe
# call of 4096 config-3-sized pairs, summed per kernel.
set -e
OUT=gpurun_out/${1:-prof_ms}
mkdir -p $OUT
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $OUT/$c -o run -- python3 tools/misscore_probe.py --pairs 4096 --reps 1 --cpu-sample 0 --check 0 --warmup 0 > $OUT/$c.log 2>&1
done
python3 - "$OUT" <<'PY'
import csv, glob, json, re, sys
out = sys.argv[1]
res = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob(f"{out}/{c}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            m = re.search(r"(\w+_kernel|\w+copyBuffer)", row["Kernel_Name"])
            k = m.group(1) if m else row["Kernel_Name"][:40]
            res.setdefault(k, {}).setdefault(c, []).append(float(row["Counter_Value"]))
summary = {}
for k, v in res.items():
    d = {c: sum(x) for c, x in v.items()}
    d["dispatches"] = max(len(x) for x in v.values())
    summary[k] = d
probe = [json.loads(l) for l in open(f"{out}/FETCH_SIZE.log") if l.startswith("{")]
print(json.dumps({"method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes; values in kB (x1024 for bytes); "
                  "FETCH_SIZE to be doubled per the gfx950 under-count (MI355X_MICROARCH.md)",
                  "kernels": summary, "probe": probe[-1] if probe else None}, indent=1))
PY
