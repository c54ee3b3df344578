"""TEST INFRASTRUCTURE: a synthetic AlnFeature workspace (SVscope.py:241-339).

pysam, bedtools, tabix and the reference's pickled random forest are not
usable here, so the AlnFeature tail is pinned on synthetic inputs:
  * per-sample alignment beds in `bedtools bamtobed -cigar` layout, served by
    FakeTabixFile (a pysam.TabixFile stand-in: fetch() / fetch(chrom, s, e));
    the .bed.gz paths exist as empty placeholders so nothing re-runs bedtools;
  * a Raw.bed with EMOutput rows whose read ids point into those beds, a
    genome-window file, InterALNSVs.vcf and a .fai;
  * StubForest: a deterministic stand-in for the random forest (predict_proba
    from |MisScore| and coverage, predict = proba > 0.5).
The workspace is rebuilt from a seed into any directory, so the reference's
code (golden generator) and this build's see identical inputs.
"""
import os

import numpy as np

CHROMS = ("chrA", "chrB")
BASES = "ACGT"


def _seq(rs, n):
    return "".join(BASES[i] for i in rs.randint(0, 4, size=n))


def _mutate(rs, s, n_edit):
    s = list(s)
    for _ in range(n_edit):
        p = rs.randint(len(s))
        op = rs.randint(3)
        if op == 0:
            s[p] = BASES[rs.randint(4)]
        elif op == 1 and len(s) > 1:
            s.pop(p)
        else:
            s.insert(p, BASES[rs.randint(4)])
    return "".join(s)


def build(seed=7):
    """Returns the workspace description: beds, raw rows, windows, inter VCF."""
    rs = np.random.RandomState(seed)
    beds = {"T1": [], "N1": []}
    raw = []
    windows = []
    n = 0
    for k in range(14):
        chrom = CHROMS[k % 2]
        ws = 10000 + 5000 * k
        we = ws + 200 + rs.randint(400)
        windows.append((chrom, ws, we))
        ids = {"T1": [], "N1": []}
        for sample, cnt in (("T1", 8 + rs.randint(6)), ("N1", 6 + rs.randint(6))):
            for _ in range(cnt):
                n += 1
                rid = "rd%05d" % n
                s = ws - rs.randint(0, 400)
                e = we + rs.randint(-100, 400)
                mq = int(rs.choice([0, 3, 20, 60, 60, 60]))
                strand = "+-"[rs.randint(2)]
                beds[sample].append((chrom, s, e, rid, mq, strand, "%dM" % (e - s)))
                if rs.random_sample() < 0.25:  # a supplementary piece elsewhere
                    oc = CHROMS[rs.randint(2)]
                    os_ = 200000 + rs.randint(50000)
                    beds[sample].append((oc, os_, os_ + 300, rid, 60, "+", "300M"))
                ids[sample].append(rid)
        base = _seq(rs, 120 + rs.randint(200))
        kind = k % 4
        if kind == 0:
            som = base[:60] + _seq(rs, 60 + rs.randint(80)) + base[60:]      # insertion >= 50
        elif kind == 1:
            som = base[:40] + base[40 + 55 + rs.randint(30):]                 # deletion <= -50
        else:
            som = _mutate(rs, base, 3 + rs.randint(8))                        # MisAlign
        som_ids = ",".join("T1_tumor|" + x for x in ids["T1"][:4])
        germ_ids = ",".join("T1_tumor|" + x for x in ids["T1"][4:]) + ";" + \
            ",".join("N1_normal|" + x for x in ids["N1"])
        germ = base + ";" + _mutate(rs, base, 2)
        if k == 5:
            som = som + ";" + _mutate(rs, som, 4)  # two somatic clusters
            som_ids = som_ids + ";" + ",".join("T1_tumor|" + x for x in ids["T1"][4:6])
        flag = "NormalOutput|EMOutput" if k % 7 != 6 else "NoEnoughspanReads"
        nsom = len(som.split(";"))
        ngerm = len(germ.split(";"))
        if flag != "NormalOutput|EMOutput":
            raw.append((chrom, ws, we, "-", "-", 0, "-", "-", 0, flag))
        else:
            raw.append((chrom, ws, we, som, som_ids, nsom, germ, germ_ids, ngerm, flag))
    for s in beds:
        beds[s].sort()
    genome = [(CHROMS[i % 2], 5000 + 3000 * i, 6000 + 3000 * i) for i in range(40)]
    inter = [("chrA", 123456, "InterALN.INS.1", "A", "AT", ".", "PASS", "SVTYPE=INS", "GT", "0/1"),
             ("chrB", 23456, "InterALN.DEL.2", "AT", "A", ".", "PASS", "SVTYPE=DEL", "GT", "0/1")]
    return {"beds": beds, "raw": raw, "windows": windows, "genome": genome, "inter": inter}


def write(workdir, seed=7):
    """Writes the workspace files; returns the paths AlnFeature's args need."""
    d = build(seed)
    os.makedirs(workdir, exist_ok=True)
    for s in d["beds"]:
        open(os.path.join(workdir, "%s.bed.gz" % s), "w").close()  # placeholder: no bamtobed re-run
    raw = os.path.join(workdir, "T1.vs.N1.TandemRepeat.Raw.bed")
    with open(raw, "w") as fh:
        for r in d["raw"]:
            fh.write("\t".join(str(x) for x in r) + "\n")
    gw = os.path.join(workdir, "genome.windows.bed")
    with open(gw, "w") as fh:
        for c, s, e in d["genome"]:
            fh.write("%s\t%d\t%d\n" % (c, s, e))
    with open(os.path.join(workdir, "InterALNSVs.vcf"), "w") as fh:
        fh.write("##fileformat=VCFv4.2\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\tT1\n")
        for r in d["inter"]:
            fh.write("\t".join(str(x) for x in r) + "\n")
    ref = os.path.join(workdir, "ref.fa")
    open(ref, "w").close()
    with open(ref + ".fai", "w") as fh:
        fh.write("chrA\t1000000\t6\t60\t61\nchrB\t800000\t1016676\t60\t61\n")
    return {"rawBedFile": raw, "genomeWindow": gw, "Reference": ref}


_CACHE = {}


def _lines(path):
    sample = os.path.basename(path).split(".")[0]
    key = (sample,)
    if key not in _CACHE:
        _CACHE[key] = ["\t".join(str(x) for x in r) for r in build()["beds"][sample]]
    return _CACHE[key]


class FakeTabixFile:
    """pysam.TabixFile stand-in over the workspace beds (path = <dir>/<sample>.bed.gz)."""

    def __init__(self, path, *a, **k):
        self.rows = _lines(path)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False

    def fetch(self, reference=None, start=None, end=None):
        for line in self.rows:
            f = line.split("\t")
            if reference is None or (f[0] == reference and int(f[1]) < end and int(f[2]) > start):
                yield line


class FakeTabixReaders:
    def tabix(self, path):
        return FakeTabixFile(path)


class StubForest:
    """Deterministic stand-in for the random forest (columns in FEATURES order)."""

    def predict_proba(self, X):
        x = np.asarray(X, dtype=float)
        z = 0.04 * x[:, 4] + 0.5 * np.nan_to_num(x[:, 0]) - 1.0
        p = 1.0 / (1.0 + np.exp(-z))
        return np.stack([1 - p, p], axis=1)

    def predict(self, X):
        return self.predict_proba(X)[:, 1] > 0.5
