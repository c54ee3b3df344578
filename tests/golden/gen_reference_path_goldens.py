"""Generates tests/golden/reference_path_goldens.json (+ reference_em_inputs.npz)
from the REFERENCE's own decision code at the BASELINE window sizes
(VERDICT r04 "next" item 1): nothing here is the builder's restatement except
the POA, which stands in for pyspoa.

Run in the build container only (needs /root/reference):
    python -B tests/golden/gen_reference_path_goldens.py [--procs 8]

Windows (synth.make_window, the generators bench.py and gen_path_goldens.py
use):
  * config3: window ids 0..15 of bench_config3_digests.json (64 reads x 3 kb);
  * config2: window ids 0..15 of config2_digests.json (32 reads x 2 kb);
  * harsh:   window ids 0..3 of harsh_digests.json (64 reads x 3 kb, 15 %
             error, 1.5-2.5 kb insertions).

Each worker imports /root/reference/src/DecisionMaker.py (-> DataScanner.py,
ReadsCluster.py) with `spoa` stubbed by this repo's C++ POA oracle and `pysam`
by an empty module, exactly as gen_decision_goldens.py does, and runs
`DecisionMaker.Decision` (what SomTDDetector.TDscope_npz:63-73 calls) after
`np.random.seed(2023)` (the per-window RNG contract).  Written per
window: the SHA-256 of the record line (the Raw.bed line of SVscope.py:171-180,
hashed as decision_oracle.record_line does) and the record's flag.

For the config-3 windows it also runs the reference's
`DataScanner.MSAFeatureSelection` and, from a fresh seed 2023,
`ReadsCluster.EMCluster(seqdatamx, initselection=1)` on the real seqdatamx the
MSA produces, and writes K, Rclust and BICList (json) and the seqdatamx itself
(npz): the EM goldens at the headline size (ReadsCluster.py:221-277).
Only inputs and outputs are written; no reference source travels.

Because the POA here is the repo's own spoa restatement, these goldens pin
the reference's decision, feature, EM and record code, not POA/consensus
parity with spoa itself, which stays unpinned (pyspoa is absent).
"""
import argparse
import hashlib
import json
import multiprocessing as mp
import os
import sys
import time
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/src"
OUT = os.path.join(HERE, "reference_path_goldens.json")
OUT_NPZ = os.path.join(HERE, "reference_em_inputs.npz")

SETS = {
    "config3": dict(n=16, reads=64, ref_len=3000, kw={}, digests="bench_config3_digests.json", em=True),
    "config2": dict(n=16, reads=32, ref_len=2000, kw={}, digests="config2_digests.json", em=False),
    "harsh": dict(n=4, reads=64, ref_len=3000, kw=dict(error=0.15, ins_range=(1500, 2501)),
                  digests="harsh_digests.json", em=False),
}

_REF = {}


def _init():
    from threadpoolctl import threadpool_limits
    threadpool_limits(1)
    sys.dont_write_bytecode = True
    sys.path.insert(0, ROOT)
    from oracle import spoa_oracle
    spoa = types.ModuleType("spoa")
    spoa.poa = spoa_oracle.poa
    sys.modules["spoa"] = spoa
    sys.modules["pysam"] = types.ModuleType("pysam")
    sys.path.insert(0, REF)
    import DecisionMaker as DM  # reference modules (this container only)
    import DataScanner as DS
    import ReadsCluster as RC
    _REF.update(DM=DM, DS=DS, RC=RC)


def _one(job):
    name, w = job
    from svscope_amd import synth
    DM, DS, RC = _REF["DM"], _REF["DS"], _REF["RC"]
    c = SETS[name]
    seqs, ids, f5, f3, rec = synth.make_window(w, c["reads"], c["ref_len"], **c["kw"])
    t0 = time.time()
    np.random.seed(2023)
    out = DM.Decision(rec, list(seqs), np.array(ids), f5, f3)
    line = "\t".join(str(x) for x in out)
    res = dict(set=name, window=w, digest=hashlib.sha256(line.encode()).hexdigest(), flag=str(out[-1]))
    em = None
    if c["em"]:
        np.random.seed(2023)
        _, dat, _ = DS.MSAFeatureSelection(list(seqs), f5, f3, np.array(ids))
        if dat.shape[0] != 0 and dat.shape[1] >= 10:
            np.random.seed(2023)
            K, _, rclust, _, _, _, bic = RC.EMCluster(dat, initselection=1)
            res.update(K=int(K), Rclust=[int(x) for x in rclust], BICList=[float(x) for x in bic],
                       nf=int(dat.shape[1]), n=int(dat.shape[0]))
            em = np.asarray(dat, dtype=np.int8)
    res["cpu_s"] = round(time.time() - t0, 1)
    return res, em


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=8)
    args = ap.parse_args()
    sys.path.insert(0, ROOT)
    from oracle import spoa_oracle
    spoa_oracle._load()
    jobs = [(name, w) for name in SETS for w in range(SETS[name]["n"])]
    # the slow (64-read) windows first
    jobs.sort(key=lambda j: -SETS[j[0]]["reads"] * SETS[j[0]]["ref_len"])
    t0 = time.time()
    with mp.get_context("fork").Pool(args.procs, initializer=_init) as pool:
        results = pool.map(_one, jobs, chunksize=1)
    results.sort(key=lambda r: (list(SETS).index(r[0]["set"]), r[0]["window"]))
    out = {
        "generator": "tests/golden/gen_reference_path_goldens.py: the reference's DecisionMaker.Decision "
                     "(spoa -> oracle POA, pysam stubbed), np.random.seed(2023) per window",
        "hash": "sha256 of the tab-joined record (decision_oracle.record_line), utf-8",
        "sets": {k: dict(reads=v["reads"], ref_len=v["ref_len"], n=v["n"], oracle_digests=v["digests"],
                         make_window_kw={a: list(b) if isinstance(b, tuple) else b for a, b in v["kw"].items()})
                 for k, v in SETS.items()},
        "windows": [r for r, _ in results],
        "cpu_s": round(time.time() - t0, 1),
    }
    with open(OUT, "w") as fh:
        json.dump(out, fh, indent=1)
    arrays = {f"{r['set']}_{r['window']}": em for r, em in results if em is not None}
    np.savez_compressed(OUT_NPZ, **arrays)
    # the reference's records against the oracle digests already committed
    mism = 0
    for r, _ in results:
        d = json.load(open(os.path.join(HERE, SETS[r["set"]]["digests"])))
        if d["digests"][r["window"]] != r["digest"]:
            mism += 1
            print("MISMATCH vs oracle digest:", r["set"], r["window"])
    print("wrote", OUT, OUT_NPZ, f"{out['cpu_s']} s", "oracle-digest mismatches:", mism)


if __name__ == "__main__":
    main()
