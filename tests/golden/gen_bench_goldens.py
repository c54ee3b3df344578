"""Generates tests/golden/bench_config3_digests.json: the CPU oracle's record
for each of bench.py's first 256 timed windows (rank 0, config 3: 64 reads x
3 kb, window ids 0..255, the SURVEY.md §8(d) generator), as the SHA-256 of
the record line (decision_oracle.record_line, the Raw.bed line format of
SVscope.py:171-180).  Digests, not lines: the fixture stays small and the
GPU test and bench.py hash their own lines the same way.

    python tests/golden/gen_bench_goldens.py [--procs 8]
    python tests/golden/gen_bench_goldens.py --sparse-stride 40   # adds ids 256, 296, ... < 10240

The sparse mode keeps the dense 0..255 digests and adds a digest for every
S-th window id after them, up to the 10,240 windows of the driver's bench
(20 steps x 512), so that bench.py's oracle_check covers every timed step.

About 25 s of CPU per window (C++ spoa restatement + numpy EM), so ~15 min on
8 cores.  Run here, in the container; only the JSON is committed.
"""
import argparse
import hashlib
import json
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

N_WINDOWS, N_READS, REF_LEN = 256, 64, 3000
OUT = os.path.join(ROOT, "tests", "golden", "bench_config3_digests.json")


def _init():
    from threadpoolctl import threadpool_limits
    threadpool_limits(1)


def _one(w):
    import numpy as np
    from svscope_amd import synth
    from oracle import decision_oracle
    r = synth.make_window(w, N_READS, REF_LEN)
    rec = decision_oracle.tdscope_npz(r[4], r[0], np.asarray(r[1]), r[2], r[3])
    line = decision_oracle.record_line(rec)
    return w, hashlib.sha256(line.encode()).hexdigest(), str(rec[-1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=8)
    ap.add_argument("--n", type=int, default=N_WINDOWS)
    ap.add_argument("--sparse-stride", type=int, default=0)
    ap.add_argument("--total", type=int, default=10240)
    args = ap.parse_args()
    from oracle import spoa_oracle
    spoa_oracle._load()
    if args.sparse_stride:
        with open(OUT) as fh:
            out = json.load(fh)
        ids = list(range(out["n"], args.total, args.sparse_stride))
        t0 = time.time()
        with mp.get_context("fork").Pool(args.procs, initializer=_init) as pool:
            res = sorted(pool.map(_one, ids, chunksize=1))
        out["sparse_ids"] = [w for w, _, _ in res]
        out["sparse_digests"] = [d for _, d, _ in res]
        out["sparse_flags"] = [f for _, _, f in res]
        out["sparse_cpu_s"] = round(time.time() - t0, 1)
        with open(OUT, "w") as fh:
            json.dump(out, fh, indent=1)
        print("wrote", OUT, len(ids), "sparse ids", f"{out['sparse_cpu_s']} s")
        return
    t0 = time.time()
    with mp.get_context("fork").Pool(args.procs, initializer=_init) as pool:
        res = sorted(pool.map(_one, range(args.n), chunksize=1))
    digests = [d for _, d, _ in res]
    out = {
        "workload": f"bench.py config 3, rank 0 window ids 0..{args.n - 1} (64 reads x 3 kb, synth.make_window)",
        "hash": "sha256 of decision_oracle.record_line(record), utf-8",
        "n": args.n,
        "digests": digests,
        "flags": [f for _, _, f in res],
        "all": hashlib.sha256("\n".join(digests).encode()).hexdigest(),
        "cpu_s": round(time.time() - t0, 1),
    }
    with open(OUT, "w") as fh:
        json.dump(out, fh, indent=1)
    print("wrote", OUT, out["all"], f"{out['cpu_s']} s")


if __name__ == "__main__":
    main()
