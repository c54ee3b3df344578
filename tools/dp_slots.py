"""LDS occupancy of the DP launches from an SVS_POA_TRACE file: each launch's
pool slots per wave (host "slots" lines, svs_poa_engine.cpp) paired in order
with its group's DP kernel lines, and the waves per SIMD its LDS allows
(160 KB per CU; kStripSlotBytes = 388 per slot per wave, svs_device.hpp),
weighted by kernel time.  The VGPR bound of the pruning instances is 7 waves
per SIMD (72 VGPRs).

  python tools/dp_slots.py trace.txt [TAIL_MS]
"""
import collections
import sys

SLOT_BYTES = 388
LDS_CU = 160 * 1024
STATIC = 256  # progress flags and per-wave scalars, bytes (upper bound)


def main(path, tail_ms=None):
    slots = collections.defaultdict(list)
    kern = collections.defaultdict(list)
    last_run = None
    for line in open(path):
        if line.startswith("# begin"):
            slots.clear()
            kern.clear()
            continue
        p = line.split()
        if not p:
            continue
        if p[0] == "host" and p[1] == "slots":
            slots[int(p[2])].append(int(p[5]))
        elif p[0] == "kern" and int(p[1]) < 10 and len(p) >= 6:
            kern[int(p[1])].append((float(p[2]), float(p[3]), int(p[5])))
    rows = []
    for g in kern:
        for (a, b, wpj), s in zip(kern[g], slots[g]):
            rows.append((a, b, wpj, s))
    if tail_ms and rows:
        end = max(r[1] for r in rows)
        rows = [r for r in rows if r[0] >= end - tail_ms]
    hist = collections.Counter()
    tot = 0.0
    for a, b, wpj, s in rows:
        lds = wpj * s * SLOT_BYTES + STATIC
        wg = LDS_CU // lds if s else 10 ** 6
        waves = min(7.0, wg * wpj / 4.0)
        hist[(wpj, s, round(waves, 2))] += b - a
        tot += b - a
    print(f"{len(rows)} DP launches, {tot:.0f} ms")
    acc = 0.0
    for k in sorted(hist, key=lambda k: -hist[k]):
        acc += hist[k]
        print(f"wpj {k[0]} slots {k[1]}: waves/SIMD {k[2]}  {hist[k]:.0f} ms ({hist[k] / tot:.1%}, cum {acc / tot:.1%})")
    w = sum(hist[k] * k[2] for k in hist) / tot if tot else 0
    print(f"time-weighted waves/SIMD allowed: {w:.2f}")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else None)
