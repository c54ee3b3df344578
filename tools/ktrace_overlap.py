"""Kernel-trace timeline summary: per kernel name total / mean time, and how
much of the wall span the DP kernel (poa_strip_kernel) and any kernel keep
the GPU busy, over the last N seconds of the trace (the timed steps).

    python tools/ktrace_overlap.py TRACE_DIR [LAST_SECONDS]
"""
import collections
import csv
import glob
import json
import os
import sys


def union(iv):
    iv = sorted(iv)
    tot, cur_s, cur_e = 0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    d = sys.argv[1]
    last = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
    rows = []
    for f in sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]))
    rows.sort()
    t_end = max(e for _, e, _ in rows)
    t0 = t_end - int(last * 1e9) if last > 0 else rows[0][0]
    rows = [x for x in rows if x[0] >= t0]
    span = t_end - rows[0][0]
    per = collections.defaultdict(list)
    for s, e, n in rows:
        per[n].append(e - s)
    out = {"span_s": span * 1e-9,
           "kernels": {n: {"count": len(v), "total_s": round(sum(v) * 1e-9, 4), "mean_ms": round(sum(v) / len(v) * 1e-6, 4)}
                       for n, v in sorted(per.items(), key=lambda kv: -sum(kv[1]))}}
    dp = [(s, e) for s, e, n in rows if "poa_strip_kernel" in n]
    out["dp_busy_frac"] = round(union(dp) / span, 4)
    out["any_busy_frac"] = round(union([(s, e) for s, e, _ in rows]) / span, 4)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
