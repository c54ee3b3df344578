"""Generates oracle digests for the localGraph paths the bench does not run
(VERDICT r03 item 4):

  * tests/golden/config2_digests.json: BASELINE.json configs[1] ("config 2"),
    32 ONT-profile reads x 2 kb, window ids 0..63 (synth.make_window);
  * tests/golden/harsh_digests.json: tools/prune_probe.py's harsh profile,
    64 reads x 3 kb at 15 % error with 1.5-2.5 kb somatic insertions, window
    ids 0..23, where the exact pruning's bound misses often and retries run.

Each is the SHA-256 of the CPU oracle's record line
(decision_oracle.record_line, the Raw.bed line of SVscope.py:171-180), as in
gen_bench_goldens.py.  Run here, in the container; only the JSON is
committed.

    python tests/golden/gen_path_goldens.py [--procs 8] [--only config2|harsh]
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

SETS = {
    "config2": dict(n=64, reads=32, ref_len=2000, kw={},
                    workload="BASELINE configs[1] (config 2): 32 reads x 2 kb, window ids 0..63, synth.make_window"),
    "harsh": dict(n=24, reads=64, ref_len=3000, kw=dict(error=0.15, ins_range=(1500, 2501)),
                  workload="tools/prune_probe.py profile: 64 reads x 3 kb, 15 % error, 1.5-2.5 kb insertions, "
                           "window ids 0..23"),
}


def _init():
    from threadpoolctl import threadpool_limits
    threadpool_limits(1)


def _one(args):
    name, w = args
    import numpy as np
    from svscope_amd import synth
    from oracle import decision_oracle
    c = SETS[name]
    r = synth.make_window(w, c["reads"], c["ref_len"], **c["kw"])
    rec = decision_oracle.tdscope_npz(r[4], r[0], np.asarray(r[1]), r[2], r[3])
    return w, hashlib.sha256(decision_oracle.record_line(rec).encode()).hexdigest(), str(rec[-1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=8)
    ap.add_argument("--only", choices=sorted(SETS))
    args = ap.parse_args()
    from oracle import spoa_oracle
    spoa_oracle._load()
    for name in ([args.only] if args.only else sorted(SETS)):
        c = SETS[name]
        t0 = time.time()
        with mp.get_context("fork").Pool(args.procs, initializer=_init) as pool:
            res = sorted(pool.map(_one, [(name, w) for w in range(c["n"])], chunksize=1))
        digests = [d for _, d, _ in res]
        out = {"workload": c["workload"], "hash": "sha256 of decision_oracle.record_line(record), utf-8",
               "reads": c["reads"], "ref_len": c["ref_len"],
               "make_window_kw": {k: list(v) if isinstance(v, tuple) else v for k, v in c["kw"].items()},
               "n": c["n"], "digests": digests, "flags": [f for _, _, f in res],
               "all": hashlib.sha256("\n".join(digests).encode()).hexdigest(), "cpu_s": round(time.time() - t0, 1)}
        path = os.path.join(ROOT, "tests", "golden", f"{name}_digests.json")
        with open(path, "w") as fh:
            json.dump(out, fh, indent=1)
        print("wrote", path, out["all"], f"{out['cpu_s']} s", flush=True)


if __name__ == "__main__":
    main()
