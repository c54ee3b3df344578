"""Compares bench.py's HIP-event DP figures with rocprofv3's kernel trace: the
mean launch duration, and the DP busy time (the union of the timed launches'
[start, end] intervals) that bench.py's roofline.frac divides by.

    python tools/rocprof_timed.py TRACE_DIR BENCH_LOG > bench_under_rocprof.json

TRACE_DIR holds the `--kernel-trace --stats --output-format csv` output of
(its kernel_trace.csv may be gzipped, as committed under profiles/)
`bench.py` run under rocprofv3; BENCH_LOG is that run's stdout (the JSON line).
bench.py times the DP launches of its timed steps only; those are the last
`poa_launches` DP dispatches of the trace, so their rocprofv3 mean is the one to
compare with bench.py's `per_launch.mean_launch_ms`, and the union of their
intervals is the one to compare with `roofline.busy_ms` (the two task groups'
launches overlap on their DP streams).
"""
import collections
import csv
import glob
import gzip
import json
import os
import sys


def union_ns(iv):
    """Total length of the union of [start, end] intervals (ns)."""
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    return tot + (cur_e - cur_s if cur_e is not None else 0)


def main():
    d, log = sys.argv[1], sys.argv[2]
    line = [l for l in open(log) if l.startswith("{")][-1]
    b = json.loads(line)
    n_timed = b["breakdown"]["poa_launches"]
    trace = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True) +
                   glob.glob(os.path.join(d, "**", "*kernel_trace.csv.gz"), recursive=True))
    rows = []
    for f in trace:
        fh = gzip.open(f, "rt") if f.endswith(".gz") else open(f)
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    per = collections.defaultdict(list)
    for s, e, name in rows:
        per[name].append((e - s) * 1e-6)
    dp = [(s, e) for s, e, name in rows if "poa_strip_kernel<" in name]
    last = dp[-n_timed:]
    rf = b["roofline"]
    mean_ms = rf["per_launch"]["mean_launch_ms"] if "per_launch" in rf else rf["mean_launch_ms"]
    bench_busy = rf["busy_ms"] if "busy_ms" in rf else rf["dp_busy"]["busy_ms"]
    busy = union_ns(last) * 1e-6
    algo = b["breakdown"]["poa_cells_computed"] * 20
    out = {
        "bench_timed_mean_launch_ms": mean_ms,
        "bench_dp_busy_ms": bench_busy,
        f"rocprof_dp_busy_ms_union_of_last_{n_timed}_launches": round(busy, 2),
        "busy_ratio_rocprof_over_bench": round(busy / bench_busy, 4) if bench_busy else None,
        "bench_frac": rf["frac"],
        "rocprof_frac_over_union": round(algo / (busy * 1e-3) / 1e9 / rf["peak"], 5) if busy else None,
        "rocprof_timed_span_ms": round((max(e for _, e in last) - min(s for s, _ in last)) * 1e-6, 2) if last else None,
        "bench_timed_launches": n_timed,
        "rocprof_dp_launches": len(dp),
        "rocprof_dp_kernel_mean_ms_all_launches_incl_warmup": round(sum(e - s for s, e in dp) * 1e-6 / max(1, len(dp)), 4),
        f"rocprof_dp_kernel_mean_ms_last_{n_timed}_launches": round(sum(e - s for s, e in last) * 1e-6 / max(1, len(last)), 4),
        "per_kernel": {k: {"calls": len(v), "mean_ms": round(sum(v) / len(v), 4), "total_ms": round(sum(v), 1)}
                       for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1]))},
        "bench_value_windows_per_s": b["value"],
        "note": f"bench.py times the {n_timed} DP launches of its timed steps with HIP events; the last {n_timed} "
                "DP dispatches of the rocprofv3 kernel trace are those launches",
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
