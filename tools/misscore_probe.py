#!/usr/bin/env python3
"""MisScore probe: N synthetic (somatic, germline) consensus pairs of config-3
size (3 kb, 2-8 % divergence, a quarter with a 100-600 bp insertion) through
svs_aligment_score_batch; prints one JSON line with GCUPS, kernel times and
the CPU oracle (C++ pairwise2 restatement) timed on a sample."""
import argparse
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def mutate(rng, a, rate, ins=0):
    b = list(a)
    for _ in range(int(len(a) * rate)):
        p, r = rng.randrange(len(b)), rng.random()
        if r < .33:
            b.pop(p)
        elif r < .66:
            b.insert(p, rng.choice("ACGT"))
        else:
            b[p] = rng.choice("ACGT")
    if ins:
        b.insert(len(b) // 2, "".join(rng.choice("ACGT") for _ in range(ins)))
    return "".join(b)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=4096)
    ap.add_argument("--len", type=int, default=3000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--cpu-sample", type=int, default=16)
    ap.add_argument("--check", type=int, default=64, help="pairs checked against the oracle")
    ap.add_argument("--warmup", type=int, default=1)
    a = ap.parse_args()
    rng = random.Random(7)
    pairs = []
    for k in range(a.pairs):
        s = "".join(rng.choice("ACGT") for _ in range(a.len))
        pairs.append((s, mutate(rng, s, rng.choice([0.02, 0.05, 0.08]), ins=rng.choice([0, 0, 0, 100, 600]))))
    from svscope_amd import _abi
    from svscope_amd.pairwise_compare import aligment_score_batch
    ctx = _abi.default_context()
    if a.warmup:
        aligment_score_batch(pairs[:64], context=ctx)
    best = None
    for _ in range(a.reps):
        st = []
        t = time.perf_counter()
        got = aligment_score_batch(pairs, context=ctx, stats=st)
        wall = time.perf_counter() - t
        s = st[0][1]
        if best is None or wall < best[0]:
            best = (wall, s)
    wall, s = best
    from oracle import pairwise2_oracle as P2
    bad = sum(got[i] != P2.AligmentScore_c(*pairs[i]) for i in range(min(a.check, len(pairs))))
    cpu = None
    if a.cpu_sample:
        t = time.perf_counter()
        for p in pairs[:a.cpu_sample]:
            P2.AligmentScore_c(*p)
        ct = time.perf_counter() - t
        cpu = {"pairs_per_s": a.cpu_sample / ct, "cores": 1, "kind": "port (C++ pairwise2 restatement, 1 thread)"}
    cells = s["dp_cells"]
    out = {"pairs": a.pairs, "len": a.len, "wall_s": round(wall, 4), "pairs_per_s": round(a.pairs / wall, 1),
           "fill_ms": round(s["fill_ms"], 3), "traceback_ms": round(s["traceback_ms"], 3),
           "fill_gcups": round(cells / (s["fill_ms"] * 1e-3) / 1e9, 2) if s["fill_ms"] else None,
           "fill_gbs_written": round(s["nib_bytes"] / (s["fill_ms"] * 1e-3) / 1e9, 2) if s["fill_ms"] else None,
           "tb_steps_per_pair": round(s["tb_steps"] / max(1, s["pairs"]), 1), "launches": s["launches"],
           "oracle_mismatches": int(bad), "checked": min(a.check, len(pairs)), "cpu": cpu}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
