"""MisScore oracle (CPU): the pairwise2 restatement against the published
examples and hand derivations (tests/golden/misscore_handchecked.json), the
C++ twin against the Python restatement, and the product's own traceback code
(misscore_tb.hpp, through tests/cpp/misscore_emu.cpp) against the oracle.
Reference: /root/reference/src/PairwiseCompare.py:19-86."""
import ctypes
import json
import os
import random
import subprocess

import pytest

from oracle import pairwise2_oracle as P2

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "misscore_handchecked.json")))
EMU_SRC = os.path.join(ROOT, "tests", "cpp", "misscore_emu.cpp")
EMU_HDR = os.path.join(ROOT, "svscope_amd", "csrc", "misscore_tb.hpp")
EMU_LIB = os.path.join(ROOT, "tests", "build", "libmisscore_emu.so")


def _emu():
    os.makedirs(os.path.dirname(EMU_LIB), exist_ok=True)
    if not os.path.exists(EMU_LIB) or os.path.getmtime(EMU_LIB) < max(os.path.getmtime(EMU_SRC),
                                                                       os.path.getmtime(EMU_HDR)):
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-o", EMU_LIB, EMU_SRC])
    lib = ctypes.CDLL(EMU_LIB)
    lib.emu_aligment_counts.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_longlong)]
    return lib


def emu_counts(lib, a, b, cutoff=0, cap=1 << 20):
    out = (ctypes.c_int * 6)()
    st = ctypes.c_longlong()
    lib.emu_aligment_counts(a.encode(), len(a), b.encode(), len(b), cutoff, cap, out, ctypes.byref(st))
    return list(out)


def random_pair(rng, max_len=30):
    alpha = rng.choice(["AC", "ACGT", "A", "ACG-", "N-", "AT"])
    a = "".join(rng.choice(alpha) for _ in range(rng.randint(1, max_len)))
    b = "".join(rng.choice(alpha) for _ in range(rng.randint(1, max_len)))
    if rng.random() < 0.5:
        b = list(a)
        for _ in range(rng.randint(0, 6)):
            op, p = rng.random(), rng.randint(0, len(b))
            if op < .3 and b:
                b.pop(min(p, len(b) - 1))
            elif op < .6:
                b.insert(p, rng.choice(alpha))
            elif b:
                b[min(p, len(b) - 1)] = rng.choice(alpha)
        b = "".join(b) or "A"
    return a, b


def mutate(rng, a, rate, ins=0):
    b = list(a)
    for _ in range(int(len(a) * rate)):
        p, r = rng.randrange(len(b)), rng.random()
        if r < .33:
            b.pop(p)
        elif r < .66:
            b.insert(p, rng.choice("ACGT"))
        else:
            b[p] = rng.choice("ACGT")
    if ins:
        b.insert(len(b) // 2, "".join(rng.choice("ACGT") for _ in range(ins)))
    return "".join(b)


@pytest.mark.parametrize("case", GOLD["order_cases"], ids=lambda c: c["source"][:40])
def test_pairwise2_order_matches_published_examples(case):
    got = P2.globalms(case["a"], case["b"], case["match"], case["mismatch"], case["open"], case["extend"])
    assert [[x, y] for x, y, _ in got] == case["alignments"]


@pytest.mark.parametrize("case", GOLD["misscore_cases"], ids=lambda c: f'{c["som"]}|{c["ger"]}|{c["cutoff"]}')
def test_misscore_hand_derived(case):
    assert P2.AligmentScore(case["som"], case["ger"], case["cutoff"]) == case["misscore"]
    assert P2.AligmentScore_c(case["som"], case["ger"], case["cutoff"]) == case["misscore"]
    n, m = emu_counts(_emu(), case["som"], case["ger"], case["cutoff"])[3:5]
    assert n - m == case["misscore"]


def test_empty_sequence_raises_like_reference():
    for c in GOLD["empty_cases"]:
        with pytest.raises(IndexError):
            P2.AligmentScore(c["som"], c["ger"])
        with pytest.raises(IndexError):
            P2.AligmentScore_c(c["som"], c["ger"])


def test_cpp_twin_matches_python_restatement():
    rng = random.Random(11)
    for _ in range(1500):
        a, b = random_pair(rng)
        cut = rng.choice([0, 0, 1, 3, 40])
        assert P2.AligmentScore(a, b, cut) == P2.AligmentScore_c(a, b, cut), (a, b, cut)


def test_product_traceback_matches_oracle_small():
    """4-bit (dh, dv) cells + misscore_tb.hpp DFS == pairwise2 restatement."""
    lib = _emu()
    rng = random.Random(12)
    for _ in range(6000):
        a, b = random_pair(rng)
        cut = rng.choice([0, 0, 1, 3, 40, 64])
        n, m, _ = P2.aligment_counts_c(a, b, cut)
        o = emu_counts(lib, a, b, cut)
        assert o[0] == 0 and (o[3], o[4]) == (n, m), (a, b, cut, (n, m), o)


def test_product_traceback_matches_oracle_3kb():
    """config-3-sized consensus pairs: 8 % divergence, with and without a
    400-bp insertion (a somatic tandem-duplication-like difference)."""
    lib = _emu()
    rng = random.Random(13)
    for k in range(6):
        a = "".join(rng.choice("ACGT") for _ in range(3000))
        b = mutate(rng, a, 0.08, ins=400 if k % 2 else 0)
        n, m, _ = P2.aligment_counts_c(a, b)
        o = emu_counts(lib, a, b)
        assert o[0] == 0 and (o[3], o[4]) == (n, m)
        assert o[5] <= 2 * (len(a) + len(b)) + 256  # the kernel's stack capacity


def test_calculate_misscore_fold_and_helpers():
    from svscope_amd import pairwise_compare as PC
    assert PC.smaller_absolute_value(3, -3) == -3 and PC.smaller_absolute_value(-2, 3) == -2
    row = {"somSeqList": "ACGTTT;AC", "germSeqList": "ACG;ACGTTTA"}
    pairs = PC._row_pairs(row)
    scores = [P2.AligmentScore(s, g) for s, g in pairs]
    assert PC._reduce(pairs, scores) == P2.CalculateMisscore(row)
    assert PC.Mismatch_abs(row) == "-1;-5"
    import pandas as pd
    td = pd.Series({"somSupportReadID": "r1_tumor,r2_tumor;r3_tumor", "germSupportReadID": "n1_normal,n2_normal;r9_tumor"})
    assert PC.CallAlleleFreq(td) == P2.CallAlleleFreq(td["somSupportReadID"], td["germSupportReadID"])
    assert PC.CallAlleleFreq(td) == "0.3333333333333333;0.16666666666666666"


def test_misscore_pipe_host_logic(tmp_path, monkeypatch):
    """MisScorePipe's parsing, filtering and per-row folds, with the alignment
    itself supplied by the oracle (the GPU path is covered in test_misscore_gpu)."""
    from svscope_amd import pairwise_compare as PC
    rows = [
        ["chr1", 100, 400, "ACGTACGT;ACG", "a_tumor,b_tumor;c_tumor", "2;1", "ACGTTCGT", "n_normal,m_normal", "2",
         "NormalOutput|EMOutput"],
        ["chr1", 500, 900, "-", "", "0", "-", "", "0", "NormalOutput"],
        ["chr2", 10, 90, "AAAA", "x_tumor", "1", "AAAAAAA;AAA", "y_normal;z_tumor", "1;1", "NormalOutput|EMOutput"],
    ]
    f = tmp_path / "x.Raw.bed"
    f.write_text("\n".join("\t".join(map(str, r)) for r in rows) + "\n")
    monkeypatch.setattr(PC, "aligment_score_batch",
                        lambda pairs, cutoff=0, context=None, stats=None: [P2.AligmentScore_c(a, b) for a, b in pairs])
    res = PC.MisScorePipe(str(f))
    assert list(res.columns) == ["chrom", "start", "end", "window", "somSupportReadID", "germSupportReadID",
                                 "MisScore", "AF"]
    assert list(res["window"]) == ["chr1_100-400", "chr2_10-90"]
    exp = [P2.CalculateMisscore({"somSeqList": r[3], "germSeqList": r[6]}) for r in (rows[0], rows[2])]
    assert list(res["MisScore"]) == exp
    assert list(res["AF"]) == [P2.CallAlleleFreq(r[4], r[7]) for r in (rows[0], rows[2])]
