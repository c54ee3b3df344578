"""Generates tests/golden/decision_goldens.json from the REFERENCE decision code.

Run in the build container only (needs /root/reference):
    python -B tests/golden/gen_decision_goldens.py

Imports /root/reference/src/DecisionMaker.py (-> DataScanner.py,
ReadsCluster.py) with two modules stubbed in sys.modules:
  * spoa  -> this repo's CPU POA oracle (pyspoa itself is not installable here:
             no network; so the POA is the oracle's, everything downstream of it
             — encoding, CallMargin, FindNonSameSite, EM, labelling, consensus
             calls, record format — is the reference's own code);
  * pysam -> an empty module (DataMaker/BAM code is not exercised).
numpy's global RNG is re-seeded with 2023 before every window (per-window RNG
contract).  Only inputs and outputs are written.
"""
import json
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/src"
OUT = os.path.join(HERE, "decision_goldens.json")


def windows():
    sys.path.insert(0, ROOT)
    from svscope_amd import synth
    out = []
    specs = [(0, 12, 500), (1, 12, 500), (2, 16, 600), (3, 16, 400), (4, 8, 700), (5, 10, 300),
             (6, 14, 500), (7, 16, 800), (8, 12, 350), (9, 10, 450)]
    for w, n, r in specs:
        out.append(("synthetic", synth.make_window(w, n, r)))
    # a full-deletion read (DataScanner.py:201-211 path)
    win = synth.make_window(10, 12, 400)
    seqs = list(win[0])
    seqs[3] = ""
    out.append(("empty_read", [seqs, win[1], win[2], win[3], win[4]]))
    # gate failures (DecisionMaker.py:134)
    win = synth.make_window(11, 8, 300)
    ids = np.array([x.replace("_tumor", "_normal") for x in win[1]])
    out.append(("one_tag", [win[0], ids, win[2], win[3], win[4]]))
    win = synth.make_window(12, 6, 300)
    out.append(("few_reads", [win[0][:3], win[1][:2], win[2], win[3], win[4]]))
    # germline-only window (no somatic haplotype among tumor reads)
    win = synth.make_window(13, 12, 500)
    seqs = [win[0][0]] + [win[0][k] if "_normal" in win[1][k - 1] else win[0][-1] for k in range(1, len(win[0]))]
    out.append(("germline_only", [seqs, win[1], win[2], win[3], win[4]]))
    # empty flanks (CallMargin quirk: DataMaker2 path passes '')
    win = synth.make_window(14, 12, 400)
    out.append(("empty_flanks", [win[0], win[1], "", "", win[4]]))
    return out


def main():
    sys.dont_write_bytecode = True
    sys.path.insert(0, ROOT)
    from oracle import spoa_oracle
    spoa = types.ModuleType("spoa")
    spoa.poa = spoa_oracle.poa
    sys.modules["spoa"] = spoa
    sys.modules["pysam"] = types.ModuleType("pysam")
    sys.path.insert(0, REF)
    import DecisionMaker as DM  # reference module (this container only)
    import DataScanner as DS

    cases = []
    for kind, (seqs, ids, f5, f3, rec) in windows():
        np.random.seed(2023)
        out = DM.Decision(rec, list(seqs), np.array(ids), f5, f3)
        np.random.seed(2023)
        feat = None
        if len(seqs) > 3:
            enc, dat, rid = DS.MSAFeatureSelection(list(seqs), f5, f3, np.array(ids))
            feat = dict(encoded_shape=list(enc.shape), seqdatamx=dat.tolist(), read_ids=list(map(str, rid)))
        cases.append(dict(kind=kind, TDRecord=rec, sequenceList=list(seqs), ReadIDs=list(map(str, ids)),
                          flank_5=f5, flank_3=f3, record=[x if isinstance(x, str) else int(x) for x in out],
                          line="\t".join(str(x) for x in out), features=feat))
        print(kind, out[-1], out[5], out[8])
    json.dump(cases, open(OUT, "w"))
    print("wrote", OUT, os.path.getsize(OUT))


if __name__ == "__main__":
    main()
