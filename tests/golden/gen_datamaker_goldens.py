"""Generates tests/golden/datamaker_goldens.json from the REFERENCE extraction
and TDscope code, over the synthetic BAM of tests/fake_bam.py.

Run in the build container only (needs /root/reference):
    python -B tests/golden/gen_datamaker_goldens.py

Imports /root/reference/src/DataScanner.py, SomTDDetector.py,
DecisionMaker.py and SomTDDetector_AimDatFetch.py with two modules stubbed in
sys.modules:
  * pysam -> AlignmentFile / FastaFile over tests/fake_bam.py's dataset (pysam
             is not installed here and no BAM fixture exists; the reads'
             aligned pairs are known by construction);
  * spoa  -> this repo's CPU POA oracle (pyspoa is not installable here).
Everything else — ReadsLoci, FetchTDsubSeq, DataMaker, ReadsLoci2,
SubSeqInWindow, DataMaker2, the AimDatFetch bundle row, Decision, EM and
TDscope's DUP re-scan — is the reference's own code.  numpy's global RNG is
re-seeded with 2023 before every Decision call (the per-window RNG contract,
DESIGN.md §3).  Only inputs (window lines; the dataset is rebuilt from its
seed) and outputs are written.
"""
import functools
import json
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/src"
OUT = os.path.join(HERE, "datamaker_goldens.json")


def _plain(x):
    if isinstance(x, np.ndarray):
        return {"ndarray": [str(v) for v in x.tolist()]}
    if isinstance(x, (list, tuple)):
        return [_plain(v) for v in x]
    if isinstance(x, (np.integer,)):
        return int(x)
    return x


def main():
    sys.dont_write_bytecode = True
    sys.path.insert(0, ROOT)
    from oracle import spoa_oracle
    from tests import fake_bam
    spoa = types.ModuleType("spoa")
    spoa.poa = spoa_oracle.poa
    sys.modules["spoa"] = spoa
    pysam = types.ModuleType("pysam")
    pysam.AlignmentFile = fake_bam.FakeAlignmentFile
    pysam.FastaFile = fake_bam.FakeFastaFile
    sys.modules["pysam"] = pysam
    sys.path.insert(0, REF)
    import DataScanner as DS  # reference modules (this container only)
    import DecisionMaker as DM
    import SomTDDetector as SD
    import SomTDDetector_AimDatFetch as AF

    refFile, bams, labels = fake_bam.paths()
    _, _, windows = fake_bam.dataset()
    off, mapq = 50, 5

    def decision(*a, **k):
        np.random.seed(2023)
        return DM.Decision(*a, **k)

    dm = functools.partial(DS.DataMaker, refFile=refFile, bamFileList=bams, LabelList=labels, offset=off, mapQ=mapq)
    dm2 = functools.partial(DS.DataMaker2, refFile=refFile, bamFileList=bams, LabelList=labels, offset=off,
                            mapQ=mapq)
    dec = functools.partial(decision, Tlabel="tumor", readcutoff=3, hcutoff=3, scutoff=0.05)
    adm = functools.partial(AF.DataMaker, refFile=refFile, bamFileList=bams, LabelList=labels, offset=off,
                            mapQ=mapq)
    cases = []
    for w in windows:
        c = {"TDRecord": w}
        c["FetchTDsubSeq"] = _plain(DS.FetchTDsubSeq(refFile, bams, labels, w, offset=off))
        c["DataMaker"] = _plain(dm(w))
        c["DataMaker2"] = _plain(dm2(w))
        chrom, start, end = w.split("\t")[0:3]
        c["SubSeqInWindow"] = _plain(DS.SubSeqInWindow(bams, labels, "\t".join([chrom, start, str(int(start) + 50)])))
        c["bundle_row"] = _plain(list(AF.TDscope(w, adm)))
        rec = SD.TDscope(w, dm, dm2, dec)
        c["TDscope"] = [x if isinstance(x, str) else int(x) for x in rec]
        c["line"] = "\t".join(str(x) for x in rec)
        cases.append(c)
        print(w.replace("\t", " "), "->", rec[-1], rec[5], rec[8])
    json.dump({"dataset": "default", "offset": off, "mapQ": mapq, "cases": cases}, open(OUT, "w"))
    print("wrote", OUT, os.path.getsize(OUT))


if __name__ == "__main__":
    main()
