#!/bin/bash
# Counters of the DP kernel instances of the driver's timed region,
# poa_strip_kernel<true, WPJ, true, unsigned short> (LDS pools, WPJ waves
# per job, pruning, 16-bit codes, single sweep) for WPJ 4, 8 and 16, on the
# driver's shape: bench.py
# with 512-window steps (--steps 4 --warmup 1).  Two SQ passes (8 counters
# each) and FETCH_SIZE / WRITE_SIZE passes, each a rocprofv3 run of its own;
# counters summed over that instance's dispatches only, and divided by the
# cells those launches evaluated (SVS_POA_TRACE: per launch its instance and
# cells computed).  Writes gpurun_out/NAME/{sq,pmc}_instance.json (one entry
# per instance; the one with the most DP time first) and pmc_dp_all.json (every
# DP dispatch: the figure profiles/pmc_poa_traffic.json carries).
#   tools/profile_instance.sh NAME [STEPS]
set -o pipefail
N=${1:?name}; STEPS=${2:-4}
OUT=gpurun_out/$N
mkdir -p $OUT
export TMPDIR=/tmp
# a counter pass serialises the kernels and prints nothing until it ends: a
# heartbeat under gpurun_out/ keeps the box from taking it for a hang
(while sleep 50; do date >> $OUT/heartbeat; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
run() {  # pass name, counters...
  local p=$1; shift
  rm -f $OUT/$p.trace
  SVS_POA_TRACE=$OUT/$p.trace timeout -s KILL 600 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$p -o run -- \
    python3 bench.py --steps $STEPS --warmup 1 --cpu-sample 0 > $OUT/$p.log 2>&1
}
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU || exit 1
run sq2 SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH || exit 1
run fetch FETCH_SIZE || exit 1
run write WRITE_SIZE || exit 1
python3 - "$OUT" "$STEPS" <<'PY'
import collections, csv, glob, json, sys
out, steps = sys.argv[1], int(sys.argv[2])


def name(wpj):
    """an instance, or (wpj None) every DP kernel instance"""
    return "poa_strip_kernel<" if wpj is None else f"poa_strip_kernel<true, {wpj}, true, unsigned short>"


def cells(p, wpj):
    """cells computed and launches of an instance (trace: kern g a b n wpj cells prune wide computed)"""
    c = n = 0
    for line in open(f"{out}/{p}.trace"):
        f = line.split()
        if f and f[0] == "kern" and len(f) >= 10 and int(f[1]) < 10 and (
                wpj is None or (f[5] == str(wpj) and f[7] == "1" and f[8] == "0")):
            c += int(f[9])
            n += 1
    return c, n


def counters(p, wpj):
    s = collections.defaultdict(float)
    disp = set()
    for f in glob.glob(f"{out}/{p}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if name(wpj) in row["Kernel_Name"]:
                s[row["Counter_Name"]] += float(row["Counter_Value"])
                disp.add((f, row.get("Dispatch_Id")))
    return dict(s), len(disp)


work = f"bench.py --steps {steps} --warmup 1 --cpu-sample 0 (512-window config-3 steps, the driver's shape)"
sq_all, pmc_all = [], []
for wpj in (4, 8, 16):
    sq, per_row, meta = {}, {}, {}
    for p in ("sq1", "sq2"):
        s, nd = counters(p, wpj)
        c, nl = cells(p, wpj)
        meta[p] = {"dispatches": nd, "launches_in_trace": nl, "cells_computed": c}
        sq.update(s)
        for k, v in s.items():
            if k.startswith("SQ_INSTS") and c:
                per_row[k] = v / (c / 64)
        if sq.get("SQ_WAVE_CYCLES"):
            per_row["wait_any_over_wave_cycles"] = sq["SQ_WAIT_ANY"] / sq["SQ_WAVE_CYCLES"]
            per_row["active_valu_over_wave_cycles"] = sq["SQ_ACTIVE_INST_VALU"] / sq["SQ_WAVE_CYCLES"]
    if not meta["sq1"]["dispatches"]:
        continue
    sq_all.append({"kernel": name(wpj), "workload": work, "per": "64-cell strip row the instance evaluated",
                   "per_strip_row": per_row, "counter_sums": sq, "passes": meta})
    f, nf = counters("fetch", wpj)
    w, nw = counters("write", wpj)
    cf, _ = cells("fetch", wpj)
    cw, _ = cells("write", wpj)
    if not (cf and cw):
        continue
    fb = f.get("FETCH_SIZE", 0.0) * 1024 * 2
    wb = w.get("WRITE_SIZE", 0.0) * 1024
    pmc_all.append({"kernel": name(wpj), "workload": work,
                    "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; kB x 1024; FETCH_SIZE "
                              "doubled (gfx950 under-count, MI355X_MICROARCH.md HBM section); this instance's dispatches only",
                    "fetch_bytes_per_cell": fb / cf, "fetch_bytes_per_cell_raw": fb / 2 / cf,
                    "write_bytes_per_cell": wb / cw, "hbm_bytes_per_cell": fb / cf + wb / cw,
                    "per": "DP cell the instance evaluated (cells_computed)",
                    "cells_computed": cf,
                    "passes": {"FETCH_SIZE": {"dispatches": nf, "cells_computed": cf},
                               "WRITE_SIZE": {"dispatches": nw, "cells_computed": cw}}})
sq_all.sort(key=lambda e: -e["counter_sums"].get("SQ_WAVE_CYCLES", 0))
pmc_all.sort(key=lambda e: -e["cells_computed"])
json.dump(sq_all, open(f"{out}/sq_instance.json", "w"), indent=1)
json.dump(pmc_all, open(f"{out}/pmc_instance.json", "w"), indent=1)
# every DP dispatch of the run (the kernel bench.py's roofline times): the
# traffic figure profiles/pmc_poa_traffic.json carries
f, nf = counters("fetch", None)
w, nw = counters("write", None)
cf, lf = cells("fetch", None)
cw, lw = cells("write", None)
fb, wb = f.get("FETCH_SIZE", 0.0) * 1024 * 2, w.get("WRITE_SIZE", 0.0) * 1024
json.dump({"kernel": "poa_strip_kernel (every instance)", "workload": work,
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; kB x 1024; FETCH_SIZE doubled "
                     "(gfx950 under-count, MI355X_MICROARCH.md HBM section); every DP dispatch of the run",
           "fetch_bytes_per_cell": fb / cf, "fetch_bytes_per_cell_raw": fb / 2 / cf, "write_bytes_per_cell": wb / cw,
           "hbm_bytes_per_cell": fb / cf + wb / cw, "per": "DP cell evaluated by the kernel (cells_computed)",
           "passes": {"FETCH_SIZE": {"kB": f.get("FETCH_SIZE", 0.0), "dispatches": nf, "cells_computed": cf, "launches": lf},
                      "WRITE_SIZE": {"kB": w.get("WRITE_SIZE", 0.0), "dispatches": nw, "cells_computed": cw,
                                     "launches": lw}}},
          open(f"{out}/pmc_dp_all.json", "w"), indent=1)
print("every DP instance: HBM B/cell", round(fb / cf + wb / cw, 3))
for e in sq_all:
    print(e["kernel"], json.dumps(e["per_strip_row"]))
for e in pmc_all:
    print(e["kernel"], "HBM B/cell", round(e["hbm_bytes_per_cell"], 3))
PY
