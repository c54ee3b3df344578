"""ORACLE — test infrastructure only.  Only tests/, __graft_entry__.smoke() and
bench-style probes import this module; the product (svscope_amd) never does.

CPU restatement of the MisScore path of the reference,
/root/reference/src/PairwiseCompare.py:

  AligmentScore        :19-30   globalms(som, ger, 1, 0, -1, -1)[0] -> middle
                                line of format_alignment -> len - count('|')
  smaller_absolute_value :32-36
  CalculateMisscore    :54-64   min-|.| over (som, ger) pairs, sign by length
  CallAlleleFreq       :66-74   (the '_tumor|' regex matches every read id)
  MisScorePipe         :76-86   rows flagged 'NormalOutput|EMOutput'

The alignment itself is third-party: Biopython's ``Bio.pairwise2`` (not
vendored under /root/reference, not pinned by its README, not installed in this
image).  It is restated here from the published Biopython >= 1.72 module
(identical in 1.72..1.81): ``_align`` on the fast path
(``_make_score_matrix_fast``: one score matrix, a 5-bit trace matrix, the
col-score vector and the on-the-fly row score), ``_find_start`` (global: the
bottom-right cell), ``_recover_alignments`` (iterative DFS with an explicit
stack, MAX_ALIGNMENTS = 1000, the no "-B over A-" rule through ``col_gap``),
``_find_gap_open``, ``_finish_backtrace``, ``_clean_alignments`` and
``format_alignment``'s match line.  Pinned by the examples printed in that
module's own docstring (tests/golden/misscore_handchecked.json) and by
hand-derived cases; everything else about pairwise2 is parity unpinned.

Pure-Python loops: meant for the small cases of the tests.  The C++ twin
(oracle/misscore_oracle.cpp, same algorithm on int matrices) covers 3 kb pairs.
"""
import re

MAX_ALIGNMENTS = 1000
_PRECISION = 1000


def rint(x, precision=_PRECISION):
    return int(x * precision + 0.5)


def calc_affine_penalty(length, open, extend, penalize_extend_when_opening):
    if length <= 0:
        return 0
    penalty = open + extend * length
    if not penalize_extend_when_opening:
        penalty -= extend
    return penalty


def _score_matrix_fast(A, B, match, mismatch, open_, extend):
    """Global, end gaps penalised, penalize_extend_when_opening False, the same
    penalties for both sequences (globalms)."""
    first_gap = calc_affine_penalty(1, open_, extend, False)
    la, lb = len(A), len(B)
    S = [[None] * (lb + 1) for _ in range(la + 1)]
    T = [[None] * (lb + 1) for _ in range(la + 1)]
    for i in range(la + 1):
        S[i][0] = calc_affine_penalty(i, open_, extend, False)
    for j in range(lb + 1):
        S[0][j] = calc_affine_penalty(j, open_, extend, False)
    col_score = [0] + [calc_affine_penalty(j, 2 * open_, extend, False) for j in range(1, lb + 1)]
    best = 0
    for r in range(1, la + 1):
        row_score = calc_affine_penalty(r, 2 * open_, extend, False)
        for c in range(1, lb + 1):
            nogap = S[r - 1][c - 1] + (match if A[r - 1] == B[c - 1] else mismatch)
            row_open = S[r][c - 1] + first_gap
            row_extend = row_score + extend
            row_score = max(row_open, row_extend)
            col_open = S[r - 1][c] + first_gap
            col_extend = col_score[c] + extend
            col_score[c] = max(col_open, col_extend)
            best = max(nogap, col_score[c], row_score)
            S[r][c] = best
            rs, cs = rint(row_score), rint(col_score[c])
            rt = (1 if rint(row_open) == rs else 0) + (8 if rint(row_extend) == rs else 0)
            ct = (4 if rint(col_open) == cs else 0) + (16 if rint(col_extend) == cs else 0)
            t = 0
            b = rint(best)
            if rint(nogap) == b:
                t += 2
            if rs == b:
                t += rt
            if cs == b:
                t += ct
            T[r][c] = t
    return S, T, best


def _finish_backtrace(A, B, sa, sb, row, col):
    if row:
        sa += A[row - 1::-1]
    if col:
        sb += B[col - 1::-1]
    if row > col:
        sb += "-" * (len(sa) - len(sb))
    elif col > row:
        sa += "-" * (len(sb) - len(sa))
    return sa, sb


def _find_gap_open(A, B, sa, sb, row, col, col_gap, S, T, stack, open_, extend, target, direction):
    dead_end = False
    target_score = S[row][col]
    for n in range(target):
        if direction == "col":
            col -= 1
            sa += "-"
            sb += B[col:col + 1]
        else:
            row -= 1
            sa += A[row:row + 1]
            sb += "-"
        actual = S[row][col] + calc_affine_penalty(n + 1, open_, extend, False)
        if rint(actual) == rint(target_score) and n > 0:
            if not T[row][col]:
                break
            stack.append((sa, sb, row, col, col_gap, T[row][col]))
        if not T[row][col]:
            dead_end = True
    return sa, sb, row, col, dead_end


def _recover(A, B, S, T, open_, extend, first_only):
    out = []
    stack = [("", "", len(A), len(B), False, T[len(A)][len(B)])]
    while stack and len(out) < MAX_ALIGNMENTS:
        dead_end = False
        sa, sb, row, col, col_gap, trace = stack.pop()
        while (row > 0 or col > 0) and not dead_end:
            cache = (sa, sb, row, col, col_gap)
            if not trace:
                if col and col_gap:
                    dead_end = True
                else:
                    sa, sb = _finish_backtrace(A, B, sa, sb, row, col)
                break
            elif trace % 2 == 1:
                trace -= 1
                if col_gap:
                    dead_end = True
                else:
                    col -= 1
                    sa += "-"
                    sb += B[col:col + 1]
                    col_gap = False
            elif trace % 4 == 2:
                trace -= 2
                row -= 1
                col -= 1
                sa += A[row:row + 1]
                sb += B[col:col + 1]
                col_gap = False
            elif trace % 8 == 4:
                trace -= 4
                row -= 1
                sa += A[row:row + 1]
                sb += "-"
                col_gap = True
            elif trace in (8, 24):
                trace -= 8
                if col_gap:
                    dead_end = True
                else:
                    col_gap = False
                    sa, sb, row, col, dead_end = _find_gap_open(
                        A, B, sa, sb, row, col, col_gap, S, T, stack, open_, extend, col, "col")
            elif trace == 16:
                trace -= 16
                col_gap = True
                sa, sb, row, col, dead_end = _find_gap_open(
                    A, B, sa, sb, row, col, col_gap, S, T, stack, open_, extend, row, "row")
            if trace:
                stack.append(cache + (trace,))
            trace = T[row][col]
        if not dead_end:
            out.append((sa[::-1], sb[::-1]))
            if first_only:
                break
    return out


def globalms(seqA, seqB, match, mismatch, open_, extend, first_only=False):
    """pairwise2.align.globalms(seqA, seqB, match, mismatch, open, extend):
    list of (alignA, alignB, score) in pairwise2's order (duplicates removed).
    first_only stops at the first recovered alignment, which is element [0] of
    the full list (the recovery appends in order and dedup keeps the first)."""
    if not seqA or not seqB:
        return []
    S, T, best = _score_matrix_fast(seqA, seqB, match, mismatch, open_, extend)
    alns = _recover(seqA, seqB, S, T, open_, extend, first_only)
    if not alns:
        # pairwise2 retries on the transposed problem (only reachable with
        # different penalties for the two sequences; kept for completeness)
        raise NotImplementedError("no alignment recovered")
    uniq = []
    for a in alns:
        if a not in uniq:
            uniq.append(a)
    return [(a, b, best) for a, b in uniq]


def match_line(alignA, alignB):
    """format_alignment(...).split('\\n')[1] for a global alignment."""
    out = []
    for a, b in zip(alignA, alignB):
        if a == b:
            out.append("|")
        elif a.strip() == "-" or b.strip() == "-":
            out.append(" ")
        else:
            out.append(".")
    return "".join(out)


def AligmentScore(SomConsensus, GerConsensus, cutoff=0):
    """PairwiseCompare.py:19-30."""
    a, b, _ = globalms(SomConsensus, GerConsensus, 1, 0, -1, -1, first_only=True)[0]
    alig = match_line(a, b)
    td = alig[cutoff:len(alig) - cutoff]
    return len(td) - td.count("|")


def smaller_absolute_value(a, b):
    """PairwiseCompare.py:32-36 (ties go to b)."""
    return a if abs(a) < abs(b) else b


def CalculateMisscore(callLine, score_fn=AligmentScore):
    """PairwiseCompare.py:54-64."""
    mis = 1000000000000000000000
    for som in callLine["somSeqList"].split(";"):
        for ger in callLine["germSeqList"].split(";"):
            s = score_fn(som, ger)
            if len(som) < len(ger):
                s = -1 * s
            mis = smaller_absolute_value(mis, s)
    return mis


def CallAlleleFreq(somSupportReadID, germSupportReadID):
    """PairwiseCompare.py:66-74 ('_tumor|' matches every id, so every germline
    read counts)."""
    import numpy as np
    som = np.array([len(x.split(",")) for x in somSupportReadID.split(";")])
    germ = np.concatenate([x.split(",") for x in germSupportReadID.split(";")])
    tumor = [x for x in germ if re.search("_tumor|", x)]
    n = np.sum(som) + len(tumor)
    return ";".join([str(x) for x in som / n])


# ---------------------------------------------------------------- C++ twin
_clib = None


def _load_c():
    global _clib
    if _clib is not None:
        return _clib
    import ctypes
    import os
    import subprocess
    here = os.path.dirname(os.path.abspath(__file__))
    path = os.path.join(here, "build", "liboracle_misscore.so")
    if not os.path.exists(path):
        subprocess.check_call(["make", "-s", "-C", here])
    lib = ctypes.CDLL(path)
    lib.oracle_aligment_counts.restype = ctypes.c_int
    lib.oracle_aligment_counts.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int] + \
        [ctypes.c_int] * 5 + [ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                              ctypes.POINTER(ctypes.c_longlong)]
    _clib = lib
    return lib


def aligment_counts_c(som, ger, cutoff=0, match=1, mismatch=0, open_=-1, extend=-1):
    """(len(TD_alig), count('|'), traceback steps) of AligmentScore's match line,
    from the C++ twin.  Raises IndexError like the reference on an empty input."""
    import ctypes
    lib = _load_c()
    a, b = som.encode("ascii"), ger.encode("ascii")
    n, m, st = ctypes.c_int(), ctypes.c_int(), ctypes.c_longlong()
    rc = lib.oracle_aligment_counts(a, len(a), b, len(b), match, mismatch, open_, extend, cutoff,
                                    ctypes.byref(n), ctypes.byref(m), ctypes.byref(st))
    if rc == -1:
        raise IndexError("list index out of range")
    if rc != 0:
        raise RuntimeError("no alignment recovered")
    return n.value, m.value, st.value


def AligmentScore_c(SomConsensus, GerConsensus, cutoff=0):
    n, m, _ = aligment_counts_c(SomConsensus, GerConsensus, cutoff)
    return n - m
