"""Generates tests/golden/big_window_digests.json: the CPU oracle's records
for windows beyond the 64-read configs: 300 tumor + 300
normal reads of 1.2 kb, and 160 + 160 reads of 2 kb (synth.make_window,
seeded), as the SHA-256 of the Raw.bed record line plus the line itself.

    python tests/golden/gen_big_window_goldens.py

A few minutes of CPU (C++ spoa restatement + numpy EM); run here, in the
container; only the JSON is committed.
"""
import hashlib
import json
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

# (window id, reads, reference length)
WINDOWS = [(7, 600, 1200), (8, 320, 2000)]
OUT = os.path.join(ROOT, "tests", "golden", "big_window_digests.json")


def _one(spec):
    import numpy as np
    from threadpoolctl import threadpool_limits
    from svscope_amd import synth
    from oracle import decision_oracle
    threadpool_limits(1)
    w, n, L = spec
    r = synth.make_window(w, n, L)
    t0 = time.time()
    rec = decision_oracle.tdscope_npz(r[4], r[0], np.asarray(r[1]), r[2], r[3])
    line = decision_oracle.record_line(rec)
    return {"window": w, "reads": n, "ref_len": L, "sha256": hashlib.sha256(line.encode()).hexdigest(),
            "flag": str(rec[-1]), "line": line, "cpu_s": round(time.time() - t0, 1)}


def main():
    with mp.get_context("fork").Pool(len(WINDOWS)) as pool:
        res = pool.map(_one, WINDOWS, chunksize=1)
    out = {"generator": "synth.make_window(window, reads, ref_len); decision_oracle.tdscope_npz",
           "hash": "sha256 of decision_oracle.record_line(record), utf-8", "windows": res}
    with open(OUT, "w") as fh:
        json.dump(out, fh, indent=1)
    print("wrote", OUT, [(r["window"], r["flag"], r["cpu_s"]) for r in res])


if __name__ == "__main__":
    main()
