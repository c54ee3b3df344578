"""DP-stream idle gaps in a rocprofv3 kernel trace: over the last N seconds,
the DP kernel's busy time, the gaps between DP launches and which other
kernels ran in them.

    python tools/gap_report.py TRACE_DIR [LAST_SECONDS]
"""
import collections
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    last = float(sys.argv[2]) if len(sys.argv) > 2 else 12.0
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]))
    rows.sort()
    dp = [(s, e) for s, e, n in rows if "poa_strip_kernel" in n]
    t0 = dp[-1][1] - last * 1e9
    dp = [x for x in dp if x[0] >= t0]
    span = dp[-1][1] - dp[0][0]
    busy = sum(e - s for s, e in dp)
    gaps = [(dp[i][1], dp[i + 1][0]) for i in range(len(dp) - 1)]
    big = [g for g in gaps if g[1] - g[0] > 1e6]
    inside = collections.Counter()
    for gs, ge in big:
        for s, e, n in rows:
            if e > gs and s < ge and "poa_strip" not in n:
                inside[n] += min(e, ge) - max(s, gs)
    hist = collections.Counter()
    for gs, ge in gaps:
        ms = (ge - gs) / 1e6
        hist["<1" if ms < 1 else "1-5" if ms < 5 else "5-15" if ms < 15 else "15-50" if ms < 50 else ">50"] += ms
    print(f"DP launches {len(dp)}, span {span / 1e9:.2f} s, DP busy {busy / 1e9:.2f} s ({busy / span:.1%}), "
          f"gaps {sum(g[1] - g[0] for g in gaps) / 1e9:.2f} s")
    print("gap ms by size:", {k: round(v, 1) for k, v in sorted(hist.items())})
    print("kernel time inside gaps > 1 ms (s):", {k[:40]: round(v / 1e9, 3) for k, v in inside.most_common(8)})


if __name__ == "__main__":
    main()
