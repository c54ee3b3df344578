"""TEST INFRASTRUCTURE: a deterministic synthetic "BAM" with the read fields
pysam exposes and the reference's extraction code reads
(/root/reference/src/DataScanner.py:57-122,249-325; SomTDDetector_AimDatFetch.py:29-105).

pysam is not installed in this image and no BAM fixture exists, so the window
extraction path is pinned on synthetic alignments whose pairs are known by
construction: FakeAlignmentFile / FakeFastaFile stand in for
pysam.AlignmentFile / pysam.FastaFile, both in svscope_amd's own extractor
(through its `readers` hook) and, in the golden generator, in the reference's
code (through a stub `pysam` module).  Paths are "fake:<dataset>:<bam-index>"
and "fake:<dataset>:ref"; the data is rebuilt from the dataset name, so bound
partials stay picklable and worker processes see the same reads.

The dataset (one chromosome, chrF) holds windows that exercise every branch
of the extractors and of TDscope's DUP re-scan:
  * a spanned window with a tumor-only insertion (EMOutput on the first call),
  * DUP windows wider than the reads (NoEnoughspanReads on the first call)
    whose 5' or 3' 50-bp corner carries a tumor-only insertion (Record5 /
    Record3), or neither (flag rewrite), or a tumor-free corner,
  * a window whose reference holds an N (GapRegion), one with too few reads,
  * reads with hard-clipped supplementary pieces (split reads), secondary
    alignments, low mapQ, N bases, and a read whose two alignments both span
    a flank (blacklisted).
"""
import functools

import numpy as np

CHROM = "chrF"
BASES = "ACGT"


class FakeRead:
    """The pysam.AlignedSegment fields the extractors read."""

    def __init__(self, name, seq, mapq, start, pairs, cigar, secondary=False, supplementary=False):
        self.query_name = name
        self.query_sequence = seq
        self.mapq = mapq
        self.mapping_quality = mapq
        self.is_secondary = secondary
        self.is_supplementary = supplementary
        self.aligned_pairs = pairs
        refs = [r for _, r in pairs if r is not None]
        self.reference_start = min(refs)
        self.reference_end = max(refs) + 1
        self.cigar = cigar
        self.cigartuples = cigar
        self.reference_name = CHROM

    @property
    def qname(self):
        return self.query_name


def _cigar(pairs, hard5=0):
    ops = []
    if hard5:
        ops.append((5, hard5))
    first = next(i for i, (q, r) in enumerate(pairs) if q is not None and r is not None)
    last = max(i for i, (q, r) in enumerate(pairs) if q is not None and r is not None)
    for i, (q, r) in enumerate(pairs):
        if q is not None and r is None:
            op = 4 if (i < first or i > last) else 1
        elif q is None:
            op = 2
        else:
            op = 0
        if ops and ops[-1][0] == op:
            ops[-1] = (op, ops[-1][1] + 1)
        else:
            ops.append((op, 1))
    return ops


def _walk(ref, rs, start, end, ins=None, dels=(), err=0.03, q0=0, nrate=0.0):
    """Reads ref[start:end] with small errors; ins: {ref pos: inserted string
    placed before it}; dels: ref ranges skipped.  Returns (bases, pairs)."""
    ins = ins or {}
    q, pairs = [], []
    for p in range(start, end):
        if p in ins:
            for b in ins[p]:
                pairs.append((q0 + len(q), None))
                q.append(b)
        if any(a <= p < b for a, b in dels):
            pairs.append((None, p))
            continue
        u = rs.random_sample()
        if u < err * 0.3 and p not in (start, end - 1):
            pairs.append((None, p))
            continue
        b = ref[p]
        if u < err * 0.7:
            b = BASES[(BASES.index(b) + 1 + rs.randint(3)) % 4]
        if rs.random_sample() < nrate:
            b = "N"
        pairs.append((q0 + len(q), p))
        q.append(b)
        if rs.random_sample() < err * 0.3 and p != end - 1:
            pairs.append((q0 + len(q), None))
            q.append(BASES[rs.randint(4)])
    return "".join(q), pairs


def _rand_seq(rs, n):
    return "".join(BASES[i] for i in rs.randint(0, 4, size=n))


class _Builder:
    def __init__(self, seed):
        self.rs = np.random.RandomState(seed)
        self.ref = list(_rand_seq(self.rs, 26000))
        self.bams = [[], []]  # tumor, normal
        self.windows = []
        self.n = 0

    def name(self, tag):
        self.n += 1
        return "%s%04d" % (tag, self.n)

    def read(self, bam, start, end, ins=None, dels=(), mapq=60, nrate=0.0, soft=(0, 0)):
        rs = self.rs
        ref = "".join(self.ref)
        seq, pairs = _walk(ref, rs, start, end, ins, dels, nrate=nrate)
        s5, s3 = _rand_seq(rs, soft[0]), _rand_seq(rs, soft[1])
        pairs = [(i, None) for i in range(soft[0])] + [(q + soft[0] if q is not None else None, r) for q, r in pairs]
        n_q = soft[0] + len(seq)
        pairs += [(n_q + i, None) for i in range(soft[1])]
        name = self.name("r")
        self.bams[bam].append(FakeRead(name, s5 + seq + s3, mapq, start, pairs, _cigar(pairs)))
        return name

    def split_read(self, bam, a0, a1, b0, b1, mid="", mapq=60):
        """A read whose first piece aligns to [a0, a1) (primary, rest soft
        clipped) and whose second piece, after `mid`, aligns to [b0, b1)
        (supplementary, hard clipped)."""
        rs = self.rs
        ref = "".join(self.ref)
        p1, pairs1 = _walk(ref, rs, a0, a1)
        p2, pairs2 = _walk(ref, rs, b0, b1)
        full = p1 + mid + p2
        tail = len(mid) + len(p2)
        prim = pairs1 + [(len(p1) + i, None) for i in range(tail)]
        name = self.name("s")
        self.bams[bam].append(FakeRead(name, full, mapq, a0, prim, _cigar(prim)))
        hard = len(p1) + len(mid)
        sup = FakeRead(name, p2, mapq, b0, pairs2, _cigar(pairs2, hard5=hard), supplementary=True)
        self.bams[bam].append(sup)
        return name

    def secondary(self, bam, start, end):
        rs = self.rs
        ref = "".join(self.ref)
        seq, pairs = _walk(ref, rs, start, end)
        name = self.name("x")
        self.bams[bam].append(FakeRead(name, seq, 0, start, pairs, _cigar(pairs), secondary=True))

    def window(self, start, end, col4):
        self.windows.append("%s\t%d\t%d\t%s" % (CHROM, start, end, col4))


def _spanned_window(B, w0, w1, off, n_t=8, n_n=7, n_som=4, extras=False):
    """Reads span [w0 - off - 30, w1 + off + 30); n_som tumor reads carry a
    90-bp insertion in the middle of the window."""
    ins = {(w0 + w1) // 2: _rand_seq(B.rs, 90)}
    a, b = w0 - off - 30, w1 + off + 30
    for i in range(n_t):
        B.read(0, a - B.rs.randint(40), b + B.rs.randint(40), ins=ins if i < n_som else None,
               soft=(B.rs.randint(20), B.rs.randint(20)), nrate=0.004 if i == 1 else 0.0)
    for i in range(n_n):
        B.read(1, a - B.rs.randint(40), b + B.rs.randint(40), mapq=3 if (extras and i == 0) else 60)
    if extras:
        # tumor split read: primary over the 5' flank into the window, then a
        # 40-bp insertion, then a supplementary piece over the 3' flank
        mid = (w0 + w1) // 2
        B.split_read(0, a, mid, mid, b, mid=_rand_seq(B.rs, 40))
        # a read both of whose alignments span the 5' flank: blacklisted
        B.split_read(1, a, b, a, w0 + 5)
        B.secondary(0, a, b)


def _dup_window(B, w0, w1, ins5, ins3, n_t=7, n_n=6, tumor_corner=True):
    """A DUP window wider than every read: reads cover the 5' corner
    [w0, w0+50) or the 3' corner [w1-50, w1) only, in the four ways
    ReadsLoci2 distinguishes (spanning, starting inside, ending inside,
    contained); tumor reads 0..3 carry a 60-bp insertion in a corner when
    ins5 / ins3 ask for one."""
    i5 = {w0 + 25: _rand_seq(B.rs, 60)} if ins5 else None
    i3 = {w1 - 25: _rand_seq(B.rs, 60)} if ins3 else None
    for corner, ins in ((w0, i5), (w1 - 50, i3)):
        for i in range(n_t if tumor_corner else 0):
            kind = 0 if i < 4 else 1 + (i - 4) % 3
            lo, hi = corner - 400 - B.rs.randint(100), corner + 50 + 400 + B.rs.randint(100)
            if kind == 1:
                lo = corner + 5
            elif kind == 2:
                hi = corner + 45
            elif kind == 3:
                lo, hi = corner + 3, corner + 48
            B.read(0, lo, hi, ins=ins if kind == 0 else None)
        for i in range(n_n):
            lo, hi = corner - 400 - B.rs.randint(100), corner + 50 + 400 + B.rs.randint(100)
            B.read(1, lo, hi)


@functools.lru_cache(maxsize=4)
def dataset(name="default"):
    """Returns (reference string, [tumor reads, normal reads], window lines)."""
    seed = {"default": 20250509}.get(name, abs(hash(name)) % (2 ** 31))
    B = _Builder(seed)
    off = 50
    # 1. spanned window, tumor-only insertion, plus split / secondary /
    #    blacklisted / low-mapQ / N-base reads
    B.window(2000, 2400, "INS,90")
    _spanned_window(B, 2000, 2400, off, extras=True)
    # 2. spanned DUP window that already reports EMOutput (no re-scan)
    B.window(4000, 4300, "DUP,300")
    _spanned_window(B, 4000, 4300, off)
    # 3-6. DUP windows no read spans; re-scan outcomes by corner content
    B.window(6000, 9000, "DUP,3000")           # 5' corner insertion -> Record5
    _dup_window(B, 6000, 9000, True, False)
    B.window(10000, 13000, "DUP,3000")         # 3' corner insertion -> Record3
    _dup_window(B, 10000, 13000, False, True)
    B.window(14000, 17000, "DUP,3000")         # no insertion -> flag rewrite
    _dup_window(B, 14000, 17000, False, False)
    B.window(18000, 21000, "DUP,3000")         # corners without tumor reads
    _dup_window(B, 18000, 21000, False, False, tumor_corner=False)
    # 7. an N in the reference window: GapRegion
    B.window(22000, 22300, "INS,10")
    _spanned_window(B, 22000, 22300, off, n_som=0)
    B.ref[22150] = "N"
    # 8. too few spanning reads
    B.window(24000, 24300, "12")
    for i in range(2):
        B.read(0, 23900, 24400)
    B.read(1, 23900, 24400)
    for bam in B.bams:
        bam.sort(key=lambda r: (r.reference_start, r.query_name, r.is_supplementary))
    return "".join(B.ref), B.bams, list(B.windows)


def _parse(path):
    _, ds, what = path.split(":")
    return ds, what


class FakeAlignmentFile:
    """pysam.AlignmentFile stand-in: fetch(contig, start, end) yields the reads
    whose aligned span overlaps [start, end), in coordinate order."""

    def __init__(self, path, *args, **kw):
        ds, what = _parse(path)
        self.reads = dataset(ds)[1][int(what)]

    def fetch(self, contig, start=None, stop=None):
        for r in self.reads:
            if r.reference_name == contig and r.reference_start < stop and r.reference_end > start:
                yield r


class FakeFastaFile:
    def __init__(self, path, *args, **kw):
        ds, _ = _parse(path)
        self.seq = dataset(ds)[0]

    def fetch(self, reference=None, start=None, end=None):
        assert reference == CHROM
        return self.seq[max(0, start):end]


class FakeReaders:
    """svscope_amd.data_maker readers hook over the fake dataset."""

    def alignment(self, path):
        return FakeAlignmentFile(path)

    def fasta(self, path):
        return FakeFastaFile(path)


def paths(ds="default"):
    """refFile, bamFileList, LabelList as SVscope.py:136-137 builds them."""
    return "fake:%s:ref" % ds, ["fake:%s:0" % ds, "fake:%s:1" % ds], ["T1_tumor", "N1_normal"]
