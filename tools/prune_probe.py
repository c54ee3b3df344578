"""Exact-pruning robustness probe: localGraph end to end (DecisionBatch) on
config-3-sized windows at a harsher error profile than SURVEY.md §8(d)'s
(default 15 % ONT-like error, 1.5-2.5 kb somatic insertions), reporting
windows/s, POA cells evaluated / full matrix, kernel time and prune retries;
--check N compares the first N windows' records with the CPU oracle."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from svscope_amd import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--windows", type=int, default=512)
ap.add_argument("--reads", type=int, default=64)
ap.add_argument("--ref-len", type=int, default=3000)
ap.add_argument("--error", type=float, default=0.15)
ap.add_argument("--ins-min", type=int, default=1500)
ap.add_argument("--ins-max", type=int, default=2501)
ap.add_argument("--check", type=int, default=0)
a = ap.parse_args()
rows = [synth.make_window(w, a.reads, a.ref_len, error=a.error, ins_range=(a.ins_min, a.ins_max))
        for w in range(a.windows)]
from svscope_amd.som_td_detector import TDscope_npz_batch  # noqa: E402
TDscope_npz_batch(rows[:2])  # context + warm-up
stats = []
t = time.time()
recs = TDscope_npz_batch(rows, stats=stats)
wall = time.time() - t
poa = dict(stats)["decision_poa"]
out = {"windows": a.windows, "error": a.error, "ins_range": [a.ins_min, a.ins_max], "wall_s": round(wall, 2),
       "windows_per_s": round(a.windows / wall, 2), "prune_retries": poa["prune_retries"],
       "cells_computed_frac": round(poa["cells_computed"] / max(1, poa["dp_cells"]), 4),
       "poa_kernel_ms": round(poa["kernel_ms"], 1), "poa_launches": poa["launches"],
       "alignments": poa["alignments"],
       "em_output": sum(1 for r in recs if str(r[-1]).endswith("|EMOutput"))}
print(json.dumps(out), flush=True)
if a.check:
    import numpy as np
    from oracle import decision_oracle
    for r, g in zip(rows[:a.check], recs):
        exp = decision_oracle.tdscope_npz(r[4], r[0], np.asarray(r[1]), r[2], r[3])
        assert decision_oracle.record_line(g) == decision_oracle.record_line(exp), r[4]
    print("oracle check ok", a.check, flush=True)
