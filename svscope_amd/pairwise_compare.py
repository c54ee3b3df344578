"""MisScore of somatic vs germline consensus sequences on MI355X.

Drop-in for /root/reference/src/PairwiseCompare.py.  Same names, arguments and
results; the Biopython global alignment behind ``AligmentScore`` runs as HIP
kernels through ``svs_aligment_score_batch`` (include/svscope.h):

  AligmentScore(SomConsensus, GerConsensus, cutoff=0)   PairwiseCompare.py:19-30
  smaller_absolute_value(a, b)                          :32-36
  Mismatch_abs(callLine)                                :38-52
  CalculateMisscore(callLine)                           :54-64
  CallAlleleFreq(SomaticTD)                             :66-74
  MisScorePipe(filepath)                                :76-86

``MisScorePipe`` and ``CalculateMisscore_batch`` send every (somatic,
germline) pair of every row to the GPU in one call instead of one Biopython
call per pair.  There is no CPU fallback: without libsvscope_hip.so or a HIP
device these functions raise.
"""
import ctypes
import re

import numpy as np

from . import _abi

_BIG = 1000000000000000000000  # PairwiseCompare.py:57


def aligment_score_batch(pairs, cutoff=0, context=None, stats=None):
    """MisScore (len(alig) - alig.count('|')) for a list of (som, ger) string
    pairs, in order.  Raises IndexError for a pair with an empty sequence,
    like ``pairwise2.align.globalms(...)[0]`` does in the reference."""
    pairs = list(pairs)
    if not pairs:
        return []
    ctx = context or _abi.default_context()
    lib = ctx.lib
    index, blobs = {}, []
    pa = np.empty(len(pairs), dtype=np.int32)
    pb = np.empty(len(pairs), dtype=np.int32)
    for p, (a, b) in enumerate(pairs):
        for arr, s in ((pa, a), (pb, b)):
            k = index.get(s)
            if k is None:
                k = index[s] = len(blobs)
                blobs.append(s.encode("ascii"))
            arr[p] = k
    starts = np.zeros(len(blobs) + 1, dtype=np.int64)
    np.cumsum([len(b) for b in blobs], out=starts[1:])
    data = b"".join(blobs)
    out_len = np.zeros(len(pairs), dtype=np.int32)
    out_match = np.zeros(len(pairs), dtype=np.int32)
    out_status = np.zeros(len(pairs), dtype=np.int32)
    st = _abi.MisscoreStats()
    rc = lib.svs_aligment_score_batch(ctx.handle, len(pairs), pa.ctypes.data, pb.ctypes.data, len(blobs),
                                      starts.ctypes.data, data, int(cutoff), out_len.ctypes.data,
                                      out_match.ctypes.data, out_status.ctypes.data, ctypes.byref(st))
    _abi.check(rc, "svs_aligment_score_batch")
    if stats is not None:
        stats.append(("misscore", st.as_dict()))
    if (out_status == _abi.MS_EMPTY).any():
        raise IndexError("list index out of range")
    return [int(x) for x in out_len - out_match]


def AligmentScore(SomConsensus, GerConsensus, cutoff=0):
    """PairwiseCompare.py:19-30: columns minus identities of the first
    globalms(som, ger, 1, 0, -1, -1) alignment's match line."""
    return aligment_score_batch([(str(SomConsensus), str(GerConsensus))], cutoff)[0]


def smaller_absolute_value(a, b):
    """PairwiseCompare.py:32-36 (ties go to b)."""
    if abs(a) < abs(b):
        return a
    return b


def Mismatch_abs(callLine):
    """PairwiseCompare.py:38-52, kept with its behaviour: the running minimum
    is never updated, so each somatic entry reports its last length difference."""
    somSeqList = callLine["somSeqList"].split(";")
    germSeqList = callLine["germSeqList"].split(";")
    Res = []
    for Som in somSeqList:
        Abs = _BIG
        AbsScore = None
        for Ger in germSeqList:
            score = len(Som) - len(Ger)
            AbsScore = smaller_absolute_value(Abs, score)
        Res.append(AbsScore)
    if len(Res) > 1:
        return ";".join(map(str, Res))
    return str(Res[0])


def _row_pairs(callLine):
    som = callLine["somSeqList"].split(";")
    ger = callLine["germSeqList"].split(";")
    return [(s, g) for s in som for g in ger]


def _reduce(pairs, scores):
    """CalculateMisscore's sign and min-|.| fold (PairwiseCompare.py:57-64)."""
    mis = _BIG
    for (s, g), score in zip(pairs, scores):
        if len(s) < len(g):
            score = (-1) * score
        mis = smaller_absolute_value(mis, score)
    return mis


def CalculateMisscore(callLine):
    """PairwiseCompare.py:54-64 for one Raw.bed row (dict or pandas row)."""
    pairs = _row_pairs(callLine)
    return _reduce(pairs, aligment_score_batch(pairs))


def CalculateMisscore_batch(callLines, context=None, stats=None):
    """CalculateMisscore over many rows with one GPU call for all their pairs."""
    per_row = [_row_pairs(r) for r in callLines]
    flat = [p for pr in per_row for p in pr]
    scores = aligment_score_batch(flat, context=context, stats=stats)
    out, k = [], 0
    for pr in per_row:
        out.append(_reduce(pr, scores[k:k + len(pr)]))
        k += len(pr)
    return out


def CallAlleleFreq(SomaticTD):
    """PairwiseCompare.py:66-74.  The reference's regex '_tumor|' matches every
    read id (the empty alternative), so every germline read is counted."""
    Raw_arr = SomaticTD[["somSupportReadID", "germSupportReadID"]].to_numpy()
    somReadCountList = np.array([len(x.split(",")) for x in Raw_arr[0].split(";")])
    germReadList = np.concatenate([x.split(",") for x in Raw_arr[1].split(";")])
    germTumorReads = [x for x in germReadList if re.search("_tumor|", x)]
    N = np.sum(somReadCountList) + len(germTumorReads)
    return ";".join([str(x) for x in somReadCountList / N])


def MisScorePipe(filepath, context=None, stats=None):
    """PairwiseCompare.py:76-86: MisScore and AF of every 'NormalOutput|EMOutput'
    row of a Raw.bed, all pairs aligned in one batched GPU call."""
    import pandas as pd
    df = pd.read_csv(filepath, sep="\t", header=None)
    df.columns = ["chrom", "start", "end", "somSeqList", "somSupportReadID", "someventCount", "germSeqList",
                  "germSupportReadID", "germeventCount", "flag"]
    somDf = df.loc[df["flag"] == "NormalOutput|EMOutput"].copy()
    cols = ["chrom", "start", "end", "window", "somSupportReadID", "germSupportReadID", "MisScore", "AF"]
    SomaticRes = pd.DataFrame(columns=cols)
    if somDf.shape[0] > 0:
        somDf["window"] = somDf["chrom"] + "_" + somDf["start"].astype("str") + "-" + somDf["end"].astype("str")
        rows = [r for _, r in somDf.iterrows()]
        somDf["MisScore"] = CalculateMisscore_batch(rows, context=context, stats=stats)
        somDf["AF"] = somDf.apply(lambda x: CallAlleleFreq(x), axis=1)
        SomaticRes = somDf[cols]
    return SomaticRes
