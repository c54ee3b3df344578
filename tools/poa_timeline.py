"""Summarise an SVS_POA_TRACE timeline (svs_poa_engine.cpp PoaTrace).

Per scheduler run: wall span, kernel-busy fraction, the GPU idle gaps between
consecutive kernels and which host phases overlapped them, and kernel rate by
launch size.  Usage: python tools/poa_timeline.py trace.txt
"""
import collections
import sys


def runs(path):
    cur = None
    for line in open(path):
        if line.startswith("# begin"):
            if cur:
                yield cur
            cur = {"host": [], "kern": []}
            continue
        p = line.split()
        if not p or cur is None:
            continue
        if p[0] == "host":
            cur["host"].append((p[1], int(p[2]), float(p[3]), float(p[4]), int(p[5])))
        elif p[0] == "kern":
            cur["kern"].append((int(p[1]), float(p[2]), float(p[3]), int(p[4]), int(p[5]), int(p[6])))
    if cur:
        yield cur


def overlap(a0, a1, b0, b1):
    return max(0.0, min(a1, b1) - max(a0, b0))


def summarise(r, idx):
    ks = sorted(r["kern"], key=lambda k: k[1])
    hs = r["host"]
    if not ks:
        print(f"run {idx}: no kernels")
        return
    end = max([k[2] for k in ks] + [h[3] for h in hs])
    busy = sum(k[2] - k[1] for k in ks)
    print(f"run {idx}: span {end:.1f} ms, {len(ks)} kernels, kernel busy {busy:.1f} ms ({100 * busy / end:.1f}%)")
    gaps = [(0.0, ks[0][1])] + [(ks[i][2], ks[i + 1][1]) for i in range(len(ks) - 1)] + [(ks[-1][2], end)]
    idle = sum(max(0.0, b - a) for a, b in gaps)
    print(f"  GPU idle {idle:.1f} ms: head {max(0.0, gaps[0][1]):.1f}, tail {max(0.0, end - ks[-1][2]):.1f}")
    by = collections.Counter()
    for a, b in gaps:
        if b <= a:
            continue
        for h in hs:
            by[h[0]] += overlap(a, b, h[2], h[3])
    print("  host phases overlapping idle gaps (ms): " + ", ".join(f"{k} {v:.1f}" for k, v in by.most_common()))
    tot = collections.Counter()
    for h in hs:
        tot[h[0]] += h[3] - h[2]
    print("  host phase totals (ms): " + ", ".join(f"{k} {v:.1f}" for k, v in tot.most_common()))
    buckets = collections.defaultdict(lambda: [0, 0.0, 0])
    for g, a, b, n, w, c in ks:
        key = 1 << max(0, (n - 1).bit_length())
        buckets[key][0] += 1
        buckets[key][1] += b - a
        buckets[key][2] += c
    print("  jobs<=  launches  kernel_ms  GCUPS")
    for key in sorted(buckets):
        n, ms, c = buckets[key]
        print(f"  {key:6d}  {n:8d}  {ms:9.1f}  {c / ms / 1e6 if ms else 0:6.1f}")
    big = sorted(gaps, key=lambda x: x[0] - x[1])[:5]
    print("  largest gaps: " + ", ".join(f"{b - a:.1f}ms@{a:.0f}" for a, b in big if b > a))


def main():
    for i, r in enumerate(runs(sys.argv[1])):
        summarise(r, i)


if __name__ == "__main__":
    main()
