"""Window extraction: BAM/FASTA -> per-window bundles for the localGraph path.

Host-side producer of the Decision inputs, with the reference's names,
arguments and return values:

  ReadsLoci         /root/reference/src/DataScanner.py:57-65
  FetchTDsubSeq     :67-122   (SomTDDetector_AimDatFetch.py:29-84 is the same)
  DataMaker         :222-247  (6-tuple with the window flag)
  ReadsLoci2        :249-265
  SubSeqInWindow    :267-295
  DataMaker2        :297-325  (the DUP corner re-scan, SomTDDetector.py:41-58)
  BundleMaker       SomTDDetector_AimDatFetch.py:86-105 + TDscope :107-123
                    (its 5-field DataMaker, returned as the DatSet row)
  save_bundles      SomTDDetector_AimDatFetch.py:159-183 (the .npz writer:
                    DatSet blocks of 8192 rows, <T>.vs.<N>.TandemRepeat.batch<k>.npz)

The reference reads BAM and FASTA through pysam.  pysam is not installed in
this image, so the readers are a hook: ``readers`` (any object with
``alignment(path)`` -> an AlignmentFile-like object with ``fetch(contig,
start, stop)`` yielding AlignedSegment-like reads, and ``fasta(path)`` -> an
object with ``fetch(reference, start, end)``).  The default is pysam, imported
when first used, so a missing pysam fails loudly at the first window.  All
functions are module level and picklable when bound with functools.partial,
as SVscope.py:152-154 binds DataMaker / DataMaker2.

This is host I/O feeding the GPU path; the
arithmetic it feeds runs in DecisionBatch.
"""
import numpy as np


class PysamReaders:
    """The reference's readers (pysam.AlignmentFile / pysam.FastaFile)."""

    def alignment(self, path):
        import pysam  # absent in this image: raises here, at the first window
        return pysam.AlignmentFile(path)

    def fasta(self, path):
        import pysam
        return pysam.FastaFile(path)


DEFAULT_READERS = PysamReaders()


def _linear_pairs(reads):
    """aligned_pairs with both positions set (DataScanner.py:60-61)."""
    return [(q, r) for q, r in reads.aligned_pairs if q is not None and r is not None]


def ReadsLoci(reads, start, end, offset=0):
    """Read positions of the last aligned base at or before ``start`` and the
    first at or after ``end``, plus ``offset`` (DataScanner.py:57-65)."""
    pairs = _linear_pairs(reads)
    s = [i for i, (_, r) in enumerate(pairs) if r <= start]
    e = [i for i, (_, r) in enumerate(pairs) if r >= end]
    if not s or not e:
        raise IndexError("index -1 is out of bounds")  # np.where(...)[0][-1] / [0] on nothing
    return [offset + pairs[s[-1]][0], offset + pairs[e[0]][0]]


def _hard_clip5(reads):
    cig = reads.cigar
    return cig[0][1] if cig[0][0] == 5 else 0


def FetchTDsubSeq(refFile, bamFileList, LabelList, TDRecord, offset=200, readers=None):
    """Flank-to-flank read subsequences of the window (DataScanner.py:67-122).
    Returns (readTDSeq, readIDList, FlankMQ)."""
    readers = readers or DEFAULT_READERS
    fields = TDRecord.strip().split("\t")
    chrom, TDStart, TDEnd = fields[0], int(fields[1]), int(fields[2])
    F5start, F5end, F3start, F3end = TDStart - offset, TDStart, TDEnd, TDEnd + offset
    readIDList, readTDSeq, FlankMQ = [], [], []
    for bamIDX in range(len(bamFileList)):
        primary = []   # [qname, query_sequence, mapq] of primary alignments
        f5, f3 = [], []  # [qname, start, end]
        for reads in readers.alignment(bamFileList[bamIDX]).fetch(chrom, TDStart, TDEnd):
            if not (reads.is_secondary or reads.is_supplementary):
                primary.append([reads.query_name, reads.query_sequence, reads.mapq])
            if reads.reference_start < F5start and reads.reference_end > F5end and not reads.is_secondary:
                off = _hard_clip5(reads) if reads.is_supplementary else 0
                f5.append([reads.qname] + ReadsLoci(reads, F5start, F5end, off))
            if reads.reference_start < F3start and reads.reference_end > F3end and not reads.is_secondary:
                off = _hard_clip5(reads) if reads.is_supplementary else 0
                f3.append([reads.qname] + ReadsLoci(reads, F3start, F3end, off))
        # names seen twice on one flank are dropped (:100-104)
        n5, c5 = np.unique([x[0] for x in f5], return_counts=True)
        n3, c3 = np.unique([x[0] for x in f3], return_counts=True)
        black = set(n5[c5 >= 2]) | set(n3[c3 >= 2])
        if len(f5) * len(f3) * len(primary) == 0:
            continue
        span = sorted(set(x[0] for x in primary) & set(x[0] for x in f5) & set(x[0] for x in f3))
        span = [x for x in span if x not in black]
        if len(span) < 3:
            continue
        # min 5' start, max 3' end per read, the primary's sequence (:111-118),
        # in sorted read-name order (np.intersect1d order, kept by the concat)
        # SeqDf.loc[spanReadIDs] then the axis-1 concat: a primary name seen
        # twice fails only when it is one of the span names (pandas'
        # InvalidIndexError); duplicates among the other primaries are ignored
        span_set = set(span)
        by_name = {}
        for name, seq, mq in primary:
            if name not in span_set:
                continue
            if name in by_name:
                raise ValueError("Reindexing only valid with uniquely valued Index objects")
            by_name[name] = (seq, mq)
        for name in span:
            st = min(x[1] for x in f5 if x[0] == name)
            en = max(x[2] for x in f3 if x[0] == name)
            seq, mq = by_name[name]
            readIDList.append(LabelList[bamIDX] + "|" + name)
            readTDSeq.append(seq[st:en].replace("N", ""))
            FlankMQ.append(int(mq))
    return readTDSeq, readIDList, FlankMQ


def _flanks(fa, TDRecord, offset):
    chrom, start, end = TDRecord.strip().split("\t")[0:3]
    flank_5 = fa.fetch(chrom, int(start) - offset, int(start)).upper()
    flank_3 = fa.fetch(chrom, int(end), int(end) + offset).upper()
    example = fa.fetch(chrom, int(start) - offset, int(end) + offset).upper()
    return flank_5, flank_3, example


def DataMaker(TDRecord, refFile, bamFileList, LabelList, offset=200, mapQ=5, readers=None):
    """Window bundle for Decision (DataScanner.py:222-247):
    (sequenceList, ReadIDs, flank_5, flank_3, TDRecord, flag)."""
    readers = readers or DEFAULT_READERS
    flag = "NormalOutput"
    readTDSeq, readIDList, FlankMQ = FetchTDsubSeq(refFile, bamFileList, LabelList, TDRecord, offset=offset,
                                                   readers=readers)
    certain = [i for i in range(len(FlankMQ)) if np.min(FlankMQ[i]) >= mapQ]
    flank_5, flank_3, example = _flanks(readers.fasta(refFile), TDRecord, offset)
    if "N" in flank_5 or "N" in flank_3 or "N" in example:
        sequenceList, ReadIDs, flag = np.array([]), np.array([]), "GapRegion"
    elif len(certain) <= 3:
        sequenceList, ReadIDs, flag = np.array([]), np.array([]), "NoEnoughspanReads"
    else:
        ReadIDs = np.array([readIDList[i] for i in certain])
        sequenceList = [example] + [readTDSeq[i] for i in certain]
    return sequenceList, ReadIDs, flank_5, flank_3, TDRecord, flag


def ReadsLoci2(reads, start, end, offset):
    """Read span inside [start, end] for reads that may start or end inside
    it (DataScanner.py:249-265; the four cases of its comments)."""
    pairs = _linear_pairs(reads)
    rs, re_ = reads.reference_start, reads.reference_end
    first_le = lambda: [i for i, (_, r) in enumerate(pairs) if r <= start][-1]  # noqa: E731
    first_ge = lambda: [i for i, (_, r) in enumerate(pairs) if r >= end][0]  # noqa: E731
    if rs < start and re_ > end:             # --|--|--
        s, e = first_le(), first_ge()
    elif start <= rs < end and re_ > end:    # | --|--
        s, e = 0, first_ge()
    elif rs < start and start < re_ <= end:  # --|-- |
        s, e = first_le(), -1
    elif rs >= start and re_ <= end:         # | -- |
        s, e = 0, -1
    else:
        raise UnboundLocalError("local variable 'startPosIDX' referenced before assignment")
    return [offset + pairs[s][0], offset + pairs[e][0]]


def SubSeqInWindow(bamFileList, LabelList, window, readers=None):
    """Every read's pieces inside a short window, concatenated in read order
    of their start (DataScanner.py:267-295).  Returns (readTDSeq, readIDList,
    FlankMQ)."""
    readers = readers or DEFAULT_READERS
    fields = window.strip().split("\t")
    chrom, Start, End = fields[0], int(fields[1]), int(fields[2])
    primary, info = {}, []
    for bamIDX in range(len(bamFileList)):
        for reads in readers.alignment(bamFileList[bamIDX]).fetch(chrom, Start, End):
            rid = LabelList[bamIDX] + "|" + reads.query_name
            if not (reads.is_secondary or reads.is_supplementary):
                primary.setdefault(rid, []).append((reads.query_sequence, reads.mapq))
            if not reads.is_secondary:
                info.append([rid] + ReadsLoci2(reads, Start, End, _hard_clip5(reads)))
    # sort_values(['readStart']) — stable here; the reference's quicksort can
    # only order two pieces of one read with the same start differently
    info.sort(key=lambda x: x[1])
    readIDList, readTDSeq, FlankMQ = [], [], []
    for rid in sorted(set(primary) & set(x[0] for x in info)):
        if len(primary[rid]) != 1:
            raise ValueError("a read with two primary alignments in the window")
        seq, mq = primary[rid][0]
        readIDList.append(rid)
        readTDSeq.append("".join(seq[s:e] for r, s, e in info if r == rid))
        FlankMQ.append(mq)
    return readTDSeq, readIDList, FlankMQ


def DataMaker2(TDRecord, refFile, bamFileList, LabelList, offset=200, mapQ=5, readers=None):
    """The two 50-bp corner windows of a DUP record (DataScanner.py:297-325):
    [[sequenceList_5, ReadIDs_5, '', '', TDRecord, flag5],
     [sequenceList_3, ReadIDs_3, '', '', TDRecord, flag3]]."""
    readers = readers or DEFAULT_READERS
    fa = readers.fasta(refFile)
    chrom, start, end = TDRecord.strip().split("\t")[0:3]
    corners = (("\t".join([chrom, start, str(int(start) + 50)]), (int(start), int(start) + 50), "UnspanedSV"),
               ("\t".join([chrom, str(int(end) - 50), end]), (int(end) - 50, int(end)), "UnspannedSV"))
    out = []
    for window, (a, b), flag in corners:
        seqs, ids, mqs = SubSeqInWindow(bamFileList, LabelList, window, readers=readers)
        certain = [i for i in range(len(mqs)) if np.min(mqs[i]) >= mapQ]
        if len(certain) <= 3:
            flag = "Unspaned+NotEnoughReads"
            sequenceList, ReadIDs = np.array([]), np.array([])
        else:
            ReadIDs = np.array([ids[i] for i in certain])
            sequenceList = [fa.fetch(chrom, a, b).upper()] + [seqs[i] for i in certain]
        out.append([sequenceList, ReadIDs, "", "", TDRecord, flag])
    return out


def BundleMaker(TDRecord, refFile, bamFileList, LabelList, offset=200, mapQ=5, readers=None):
    """One DatSet row, np.array([sequenceList, ReadIDs, flank_5, flank_3,
    TDRecord], dtype=object), as SomTDDetector_AimDatFetch.py:86-123 builds
    it (its DataMaker merges GapRegion and NoEnoughspanReads: empty lists)."""
    readers = readers or DEFAULT_READERS
    readTDSeq, readIDList, FlankMQ = FetchTDsubSeq(refFile, bamFileList, LabelList, TDRecord, offset=offset,
                                                   readers=readers)
    certain = [i for i in range(len(FlankMQ)) if np.min(FlankMQ[i]) >= mapQ]
    flank_5, flank_3, example = _flanks(readers.fasta(refFile), TDRecord, offset)
    if "N" in flank_5 or "N" in flank_3 or "N" in example or len(certain) <= 3:
        sequenceList, ReadIDs = np.array([]), np.array([])
    else:
        ReadIDs = np.array([readIDList[i] for i in certain])
        sequenceList = [example] + [readTDSeq[i] for i in certain]
    return np.array([sequenceList, ReadIDs, flank_5, flank_3, TDRecord], dtype=object)


def bundle_name(TsampleID, NsampleID, batch):
    return "%s.vs.%s.TandemRepeat.batch%s.npz" % ("-".join(TsampleID), "-".join(NsampleID), batch)


def save_bundles(rows, savedir, TsampleID, NsampleID, block=8192):
    """Writes DatSet rows in blocks of ``block`` (SomTDDetector_AimDatFetch.py:
    160-183): np.savez(<savedir>/<T>.vs.<N>.TandemRepeat.batch<k>.npz,
    DatSet=np.array(rows)).  Returns the paths written."""
    import os
    paths, batch, pending = [], 0, []

    def flush():
        nonlocal batch, pending
        path = os.path.join(savedir, bundle_name(TsampleID, NsampleID, batch))
        arr = np.empty((len(pending), 5), dtype=object)
        for i, r in enumerate(pending):
            arr[i, :] = list(r)  # np.array(batch_List) of (5,) object rows
        np.savez(path, DatSet=arr)
        paths.append(path)
        pending = []
        batch += 1

    for row in rows:
        if row.shape[0] > 0:
            pending.append(row)
            if len(pending) >= block:
                flush()
    if pending:
        flush()
    return paths
