#!/bin/bash
# Counters of the DP kernel (poa_strip_kernel) over the TIMED region of the
# driver's bench command (bench.py --steps STEPS --warmup WARMUP, default 20 and
# 5: 512-window config-3 steps), per kernel instance
# (poa_strip_kernel<LDS pools, WPJ waves per job, pruning, code type>).  Two SQ
# passes (8 counters each) and FETCH_SIZE / WRITE_SIZE passes, each a rocprofv3
# run of its own.  A pass's timed DP dispatches are its last N
# poa_strip_kernel dispatches, N = the bench line's poa_launches, and the last
# N DP launches of the SVS_POA_TRACE timeline give the cells each instance
# evaluated (the two DP streams finish out of issue order, so the two lists
# are matched per instance, not launch by launch).  Counters are summed per
# instance over those dispatches only and divided by the instance's cells.
# Writes gpurun_out/NAME/{sq,pmc}_instance.json (one entry per instance, the
# one with the most timed dispatches first) and pmc_dp_all.json (every timed
# DP dispatch: the figure profiles/pmc_poa_traffic.json carries).
#   tools/profile_instance.sh NAME [STEPS] [WARMUP]
# PASSES="sq1 sq2" (or "fetch write") runs those passes only (a call's time
# limit holds two of them); the summary is written once all four are there.
set -o pipefail
N=${1:?name}; STEPS=${2:-20}; WARM=${3:-5}
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
  SVS_POA_TRACE=$OUT/$p.trace timeout -s KILL 900 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$p -o run -- \
    python3 bench.py --steps $STEPS --warmup $WARM --cpu-sample 0 > $OUT/$p.json 2> $OUT/$p.err
}
PASSES=${PASSES:-sq1 sq2 fetch write}
want() { [[ " $PASSES " == *" $1 "* ]]; }
if want sq1; then run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU || exit 1; fi
if want sq2; then run sq2 SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH || exit 1; fi
if want fetch; then run fetch FETCH_SIZE || exit 1; fi
if want write; then run write WRITE_SIZE || exit 1; fi
for p in sq1 sq2 fetch write; do [ -s $OUT/$p.json ] || { echo "passes so far: $PASSES"; exit 0; }; done
python3 - "$OUT" "$STEPS" "$WARM" <<'PY'
import collections, csv, glob, json, re, sys
out, steps, warm = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
work = (f"bench.py --steps {steps} --warmup {warm} --cpu-sample 0 (512-window config-3 steps, the driver's shape); "
        f"timed-region DP dispatches only")


NAME = re.compile(r"poa_strip_kernel<(true|false), (\d+), (true|false), unsigned (short|int)>")


def timed(p):
    """[(instance, cells computed, counters)] per instance of the pass's timed DP
    dispatches: (instance, its cells, its counter sums, dispatches counted,
    launches in the trace)"""
    n = json.load(open(f"{out}/{p}.json"))["breakdown"]["poa_launches"]
    kern = []
    for line in open(f"{out}/{p}.trace"):
        f = line.split()
        if f and f[0] == "kern" and len(f) >= 10 and int(f[1]) < 10:
            kern.append(f)
    disp = collections.OrderedDict()
    for fn in glob.glob(f"{out}/{p}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(fn)):
            if "poa_strip_kernel<" in row["Kernel_Name"]:
                d = disp.setdefault(int(row["Dispatch_Id"]), {"name": row["Kernel_Name"], "c": {}})
                d["c"][row["Counter_Name"]] = d["c"].get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    ids = sorted(disp)[-n:]
    kern = kern[-n:]
    assert len(ids) == n and len(kern) == n, (p, n, len(ids), len(kern))
    cells = collections.Counter()
    launches = collections.Counter()
    for f in kern:
        inst = f"poa_strip_kernel<wpj {f[5]}, prune {f[7]}, wide {f[8]}>"
        cells[inst] += int(f[9])
        launches[inst] += 1
    sums = collections.defaultdict(dict)
    count = collections.Counter()
    for i in ids:
        m = NAME.search(disp[i]["name"])
        assert m, disp[i]["name"]
        inst = f"poa_strip_kernel<wpj {m.group(2)}, prune {int(m.group(3) == 'true')}, wide {int(m.group(4) == 'int')}>"
        count[inst] += 1
        for k, v in disp[i]["c"].items():
            sums[inst][k] = sums[inst].get(k, 0.0) + v
    return [(inst, cells[inst], sums[inst], count[inst], launches[inst]) for inst in launches]


passes = {p: timed(p) for p in ("sq1", "sq2", "fetch", "write")}
insts = collections.Counter({i: nd for i, _, _, nd, _ in passes["sq1"]})
match = {p: {i: [nd, nl] for i, _, _, nd, nl in passes[p]} for p in passes}
passes = {p: [(i, c, s) for i, c, s, _, _ in v] for p, v in passes.items()}
sq_all, pmc_all = [], []
for inst, nd in insts.most_common():
    sq, per_row, meta = {}, {}, {}
    for p in ("sq1", "sq2"):
        c = sum(x for i, x, _ in passes[p] if i == inst)
        for i, _, cs in passes[p]:
            if i == inst:
                for k, v in cs.items():
                    sq[k] = sq.get(k, 0.0) + v
        meta[p] = {"dispatches": match[p].get(inst, [0])[0], "cells_computed": c}
        for k in list(sq):
            if k.startswith("SQ_INSTS") and c and k not in per_row:
                per_row[k] = sq[k] / (c / 64)
    if sq.get("SQ_WAVE_CYCLES"):
        per_row["wait_any_over_wave_cycles"] = sq["SQ_WAIT_ANY"] / sq["SQ_WAVE_CYCLES"]
        per_row["active_valu_over_wave_cycles"] = sq["SQ_ACTIVE_INST_VALU"] / sq["SQ_WAVE_CYCLES"]
    sq_all.append({"kernel": inst, "workload": work, "per": "64-cell strip row the instance evaluated",
                   "timed_dispatches": nd, "share_of_timed_dispatches": nd / sum(insts.values()),
                   "dispatches_vs_trace_launches": {p: match[p].get(inst) for p in match},
                   "per_strip_row": per_row, "counter_sums": sq, "passes": meta})
    fb = sum(cs.get("FETCH_SIZE", 0.0) for i, _, cs in passes["fetch"] if i == inst) * 1024 * 2
    wb = sum(cs.get("WRITE_SIZE", 0.0) for i, _, cs in passes["write"] if i == inst) * 1024
    cf = sum(x for i, x, _ in passes["fetch"] if i == inst)
    cw = sum(x for i, x, _ in passes["write"] if i == inst)
    if cf and cw:
        pmc_all.append({"kernel": inst, "workload": work,
                        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; kB x 1024; "
                                  "FETCH_SIZE doubled (gfx950 under-count, MI355X_MICROARCH.md HBM section); this "
                                  "instance's timed dispatches only",
                        "fetch_bytes_per_cell": fb / cf, "fetch_bytes_per_cell_raw": fb / 2 / cf,
                        "write_bytes_per_cell": wb / cw, "hbm_bytes_per_cell": fb / cf + wb / cw,
                        "per": "DP cell the instance evaluated (cells_computed)", "cells_computed": cf,
                        "timed_dispatches": nd})
json.dump(sq_all, open(f"{out}/sq_instance.json", "w"), indent=1)
json.dump(pmc_all, open(f"{out}/pmc_instance.json", "w"), indent=1)
# every timed DP dispatch, instance-weighted by the run's own mix: the figure
# profiles/pmc_poa_traffic.json carries (bench.py's roofline traffic)
fb = sum(cs.get("FETCH_SIZE", 0.0) for _, _, cs in passes["fetch"]) * 1024 * 2
wb = sum(cs.get("WRITE_SIZE", 0.0) for _, _, cs in passes["write"]) * 1024
cf = sum(x for _, x, _ in passes["fetch"])
cw = sum(x for _, x, _ in passes["write"])
json.dump({"kernel": "poa_strip_kernel (every instance, timed dispatches)", "workload": work,
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; kB x 1024; FETCH_SIZE doubled "
                     "(gfx950 under-count, MI355X_MICROARCH.md HBM section); the timed region's DP dispatches",
           "fetch_bytes_per_cell": fb / cf, "fetch_bytes_per_cell_raw": fb / 2 / cf, "write_bytes_per_cell": wb / cw,
           "hbm_bytes_per_cell": fb / cf + wb / cw, "per": "DP cell evaluated by the kernel (cells_computed)",
           "instances": {i: n for i, n in insts.most_common()},
           "passes": {"FETCH_SIZE": {"dispatches": sum(v[0] for v in match["fetch"].values()), "cells_computed": cf},
                      "WRITE_SIZE": {"dispatches": sum(v[0] for v in match["write"].values()), "cells_computed": cw}}},
          open(f"{out}/pmc_dp_all.json", "w"), indent=1)
print("timed DP dispatches: HBM B/cell", round(fb / cf + wb / cw, 3), dict(insts))
for e in sq_all:
    print(e["kernel"], e["timed_dispatches"], json.dumps(e["per_strip_row"]))
for e in pmc_all:
    print(e["kernel"], "HBM B/cell", round(e["hbm_bytes_per_cell"], 3), "write", round(e["write_bytes_per_cell"], 3))
PY
# the raw counter CSVs are far larger than what gpurun copies back
rm -rf $OUT/sq1 $OUT/sq2 $OUT/fetch $OUT/write
gzip -f $OUT/*.trace
