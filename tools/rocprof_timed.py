"""Compares bench.py's HIP-event DP-kernel mean with rocprofv3's kernel trace.

    python tools/rocprof_timed.py TRACE_DIR BENCH_LOG > bench_under_rocprof.json

TRACE_DIR holds the `--kernel-trace --stats --output-format csv` output of
`bench.py` run under rocprofv3; BENCH_LOG is that run's stdout (the JSON line).
bench.py times the DP launches of its timed steps only; those are the last
`poa_launches` DP dispatches of the trace, so their rocprofv3 mean is the one to
compare with bench.py's `mean_launch_ms`.
"""
import collections
import csv
import glob
import json
import os
import sys


def main():
    d, log = sys.argv[1], sys.argv[2]
    line = [l for l in open(log) if l.startswith("{")][-1]
    b = json.loads(line)
    n_timed = b["breakdown"]["poa_launches"]
    trace = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True))
    rows = []
    for f in trace:
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    per = collections.defaultdict(list)
    for s, e, name in rows:
        per[name].append((e - s) * 1e-6)
    dp = [(s, e) for s, e, name in rows if "poa_strip_kernel<" in name]
    last = dp[-n_timed:]
    out = {
        "bench_timed_mean_launch_ms": b["roofline"]["mean_launch_ms"],
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
