"""MSA encoding and feature selection (the MSA half of the per-window path).

Same names, arguments and results as /root/reference/src/DataScanner.py:
  SeqEncoder :124-129   A,T,C,G,- -> 0,1,2,3,4 (case-insensitive; KeyError otherwise)
  SeqDecoder :131-137   drops code 4
  CallMargin :146-165   reference-flank MSA columns (literal walk semantics,
                        including the empty-flank quirk), vectorised
  FindNonSameSite :167-179   columns whose second-largest symbol count >= cutoff
  MSAFeatureSelection :181-220  poa([ref]+reads, 1) -> encode -> drop flanks ->
                        informative columns; keeps the full-deletion-read
                        behaviour of :201-211 (ids of non-empty reads listed twice)
The POA runs on MI355X through svscope_amd.poa; msa_feature_selection_batch
feeds many windows through one batched GPU POA.
"""
import numpy as np

from .poa import poa_batch

_LUT = np.full(256, 255, dtype=np.uint8)
for _ch, _code in (("A", 0), ("T", 1), ("C", 2), ("G", 3), ("-", 4)):
    _LUT[ord(_ch)] = _code
    _LUT[ord(_ch.lower())] = _code
_DECODE = np.frombuffer(b"ATCG", dtype=np.uint8)


def _encode_rows(rows):
    """Encodes equal-length MSA rows into an (R, C) int64 matrix."""
    if not rows:
        return np.zeros((0, 0), dtype=np.int64)
    width = len(rows[0])
    buf = np.frombuffer("".join(rows).encode("latin-1"), dtype=np.uint8)
    codes = _LUT[buf]
    if (codes == 255).any():
        bad = buf[np.argmax(codes == 255)]
        raise KeyError(chr(bad).upper())
    return codes.astype(np.int64).reshape(len(rows), width)


def SeqEncoder(seqinput):
    return _encode_rows(["".join(seqinput)])[0] if len(seqinput) else np.array([])


def SeqDecoder(seqinput):
    a = np.asarray(seqinput)
    a = a[a != 4]
    return _DECODE[a.astype(np.int64)].tobytes().decode("ascii") if a.size else ""


def CallMargin(msa, flank_5, flank_3):
    ex = "".join(msa[0])
    arr = np.frombuffer(ex.encode("latin-1"), dtype=np.uint8)
    gap = ord("-")
    nongap = np.flatnonzero(arr != gap)
    # forward walk (:150-157): stops right after the ungapped prefix equals flank_5
    k5 = len(flank_5)
    if k5 == 0:
        part1 = nongap if (arr.size and arr[0] != gap) else nongap[:0]
    elif arr[nongap[:k5]].tobytes() == flank_5.encode("latin-1") and nongap.size >= k5:
        part1 = nongap[:k5]
    else:
        part1 = nongap
    # backward walk over indices len-1 .. 1 (:158-164)
    cand = nongap[nongap >= 1][::-1]
    k3 = len(flank_3)
    if k3 == 0:
        part2 = cand if (arr.size > 1 and arr[-1] != gap) else cand[:0]
    elif cand.size >= k3 and arr[cand[:k3][::-1]].tobytes() == flank_3.encode("latin-1"):
        part2 = cand[:k3]
    else:
        part2 = cand
    return np.concatenate([part1, part2]) if (part1.size or part2.size) else np.array([])


def FindNonSameSite(seqencode_New_Sub, cutoff=3):
    M = np.asarray(seqencode_New_Sub)
    counts = np.stack([(M == a).sum(axis=0) for a in range(5)]).astype(np.float64)
    return np.where(np.sort(counts, axis=0)[-2] >= cutoff)[0]


def _select(msa, flank_5, flank_3, read_ids, n_reads_total, seq_lens, hcutoff, scutoff):
    read_ids = np.asarray(read_ids)
    dels = np.where(seq_lens == 0)[0]
    if dels.shape[0] > 0:
        undel = np.setdiff1d(np.arange(len(read_ids)), dels)
        keep = list(read_ids[undel])
        enc = _encode_rows(msa)
        width = enc.shape[1]
        read_ids = np.array(keep + keep)
        encoded = np.vstack([enc, np.full((len(keep), width), 4, dtype=np.int64)])
        msa_rows = list(msa) + ["-" * width] * len(keep)
    else:
        encoded = _encode_rows(msa)
        msa_rows = msa
    pool = CallMargin(msa_rows, flank_5, flank_3)
    raw = encoded[1:, np.setdiff1d(np.arange(encoded.shape[1]), pool)]
    feat = raw[:, FindNonSameSite(raw, cutoff=max([hcutoff, encoded.shape[0] * scutoff]))]
    return encoded, feat, read_ids


def msa_feature_selection_batch(items, hcutoff=3, scutoff=0.05, context=None, stats=None):
    """items: list of (sequenceList, flank_5, flank_3, readIDList).
    Returns [(seqencode_New, seqdatamx, readIDList)] — one batched GPU POA."""
    if not items:
        return []
    res = poa_batch([list(it[0]) for it in items], algorithm=1, genmsa=True, context=context,
                    return_stats=stats is not None)
    if stats is not None:
        res, st = res
        stats.append(("msa_poa", st))
    out = []
    for (seqs, f5, f3, ids), (_, msa) in zip(items, res):
        lens = np.array([len(x) for x in list(seqs)[1:]])
        out.append(_select(msa, f5, f3, ids, len(seqs) - 1, lens, hcutoff, scutoff))
    return out


def MSAFeatureSelection(sequenceList, flank_5, flank_3, readIDList, hcutoff=3, scutoff=0.05):
    return msa_feature_selection_batch([(sequenceList, flank_5, flank_3, readIDList)], hcutoff, scutoff)[0]
