"""Generates tests/golden/alnfeature_goldens.json from the REFERENCE AlnFeature
(SVscope.py:241-339, DataScanner.py:328-481, OutVCF.py, PairwiseCompare.py)
over the synthetic workspace of tests/fake_tabix.py.

Run in the build container only (needs /root/reference):
    LC_ALL=C python -B tests/golden/gen_alnfeature_goldens.py

Stubbed in sys.modules (none of these is installed or usable here):
  * pysam       -> FakeTabixFile over the workspace beds (AlignmentFile and
                   FastaFile are never reached on this path);
  * Bio         -> Seq = str, pairwise2.align.globalms = this repo's restatement
                   of Biopython's pairwise2 (oracle/pairwise2_oracle.py) and a
                   format_alignment whose second line is its match line;
  * statsmodels -> an empty module (imported, never used);
  * spoa        -> the CPU POA oracle (imported by DataScanner, unused here).
SVscope.load (joblib) is replaced by tests/fake_tabix.StubForest: the
reference's model file is a pickle and is never deserialised.  The shell
steps the reference runs (grep, sort, rm) run for real with LC_ALL=C.
Only inputs (the workspace is rebuilt from its seed) and outputs are written;
the VCF ##fileDate line is dropped.
"""
import json
import os
import sys
import tempfile
import types
from types import SimpleNamespace

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/src"
OUT = os.path.join(HERE, "alnfeature_goldens.json")


def _stubs():
    from oracle import pairwise2_oracle as pw
    from oracle import spoa_oracle
    from tests import fake_tabix
    spoa = types.ModuleType("spoa")
    spoa.poa = spoa_oracle.poa
    pysam = types.ModuleType("pysam")
    pysam.TabixFile = fake_tabix.FakeTabixFile
    bio = types.ModuleType("Bio")
    seq = types.ModuleType("Bio.Seq")
    seq.Seq = str
    p2 = types.ModuleType("Bio.pairwise2")
    p2.align = types.SimpleNamespace(globalms=lambda a, b, m, mm, o, e: pw.globalms(a, b, m, mm, o, e))
    p2.format_alignment = lambda a, b, score, *rest: "%s\n%s\n%s\n  Score=%s\n" % (a, pw.match_line(a, b), b, score)
    bio.Seq, bio.pairwise2 = seq, p2
    sm = types.ModuleType("statsmodels")
    sms = types.ModuleType("statsmodels.stats")
    sms.multitest = types.ModuleType("statsmodels.stats.multitest")
    sm.stats = sms
    sys.modules.update({"spoa": spoa, "pysam": pysam, "Bio": bio, "Bio.Seq": seq, "Bio.pairwise2": p2,
                        "statsmodels": sm, "statsmodels.stats": sms,
                        "statsmodels.stats.multitest": sms.multitest})
    return fake_tabix


def _no_date(text):
    return "".join(x for x in text.splitlines(True) if not x.startswith("##fileDate"))


def main():
    sys.dont_write_bytecode = True
    sys.path.insert(0, ROOT)
    fake_tabix = _stubs()
    sys.path.insert(0, REF)
    import DataScanner as DS  # reference modules (this container only)
    import SVscope as SV
    SV.load = lambda path: fake_tabix.StubForest()
    out = {"seed": 7}
    with tempfile.TemporaryDirectory() as wd:
        paths = fake_tabix.write(wd)
        args = SimpleNamespace(savedir=wd, TSampleID="T1", NSampleID="N1", Tumorbam="t.bam", Normalbam="n.bam",
                               thread="2", **paths)
        merged = SV.AlnFeature(args)
        for name in ("T1.Somatic.bed", "RandomForestResult.tsv"):
            out[name] = open(os.path.join(wd, name)).read()
        out["T1.vcf"] = _no_date(open(os.path.join(wd, "T1.vcf")).read())
        out["T1.mergedSomatic.vcf"] = _no_date(open(merged).read())
        tbed, nbed = os.path.join(wd, "T1.bed.gz"), os.path.join(wd, "N1.bed.gz")
        db_t = os.path.join(wd, "Tumor.sqlite")
        bg = DS.background(paths["genomeWindow"], tbed, db_t, showchromSpan=False, workthread=1)
        sv = DS.background(paths["rawBedFile"], nbed, os.path.join(wd, "Normal.sqlite"), showchromSpan=True,
                           workthread=1)
        out["background_T_genome"] = json.loads(bg.to_json(orient="split"))
        out["background_N_raw"] = json.loads(sv.to_json(orient="split"))
        out["query_reads"] = [list(x) for x in DS.query_reads(db_t, "rd00003")]
        out["OVLEN"] = [[w, s, e, DS.OVLEN(w, s, e)] for w, s, e in
                        [("c\t100\t200", a, b) for a, b in ((50, 250), (120, 150), (150, 250), (50, 150),
                                                            (100, 200), (100, 150), (150, 200), (50, 100))]]
    json.dump(out, open(OUT, "w"), indent=0)
    print("wrote", OUT, os.path.getsize(OUT))


if __name__ == "__main__":
    main()
