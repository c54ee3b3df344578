"""MisScore on the GPU (svs_aligment_score_batch through svscope_amd.pairwise_compare)
against the CPU oracle (oracle/pairwise2_oracle.py + its C++ twin), bit-exact
on the match-line counts.  Reference: /root/reference/src/PairwiseCompare.py:19-86."""
import json
import os
import random

import pytest

from oracle import pairwise2_oracle as P2
from tests.test_misscore_oracle import GOLD, mutate, random_pair

pytestmark = pytest.mark.gpu


def _pc():
    from svscope_amd import pairwise_compare as PC
    return PC


def test_golden_cases(gpu_ctx):
    PC = _pc()
    for c in GOLD["misscore_cases"]:
        assert PC.AligmentScore(c["som"], c["ger"], c["cutoff"]) == c["misscore"], c
    for c in GOLD["empty_cases"]:
        with pytest.raises(IndexError):
            PC.AligmentScore(c["som"], c["ger"])


def test_random_small_pairs_one_batch(gpu_ctx):
    PC = _pc()
    rng = random.Random(21)
    pairs = [random_pair(rng) for _ in range(3000)]
    for cut in (0, 1, 64):
        got = PC.aligment_score_batch(pairs, cutoff=cut, context=gpu_ctx)
        exp = [P2.AligmentScore_c(a, b, cut) for a, b in pairs]
        bad = [(i, pairs[i], got[i], exp[i]) for i in range(len(pairs)) if got[i] != exp[i]]
        assert not bad, bad[:5]


def test_strip_and_chunk_boundaries(gpu_ctx):
    """lengths around the 64-column strips, the 64-row chunks and the 8-step
    nibble words; very unequal lengths; identical sequences."""
    PC = _pc()
    rng = random.Random(22)
    lens = [1, 2, 7, 8, 9, 62, 63, 64, 65, 66, 127, 128, 129, 191, 192, 193, 255, 256, 257]
    pairs = []
    for la in lens:
        for lb in lens:
            a = "".join(rng.choice("ACGT") for _ in range(la))
            b = mutate(rng, a, 0.1)[:lb] if lb <= la else (a + "".join(rng.choice("ACGT") for _ in range(lb - la)))
            b = b or "A"
            pairs.append((a, b))
    pairs += [("A" * 3000, "A"), ("C", "ACGT" * 700), ("ACGT" * 500, "ACGT" * 500), ("-", "ACGT" * 100)]
    got = PC.aligment_score_batch(pairs, context=gpu_ctx)
    exp = [P2.AligmentScore_c(a, b) for a, b in pairs]
    bad = [(len(pairs[i][0]), len(pairs[i][1]), got[i], exp[i]) for i in range(len(pairs)) if got[i] != exp[i]]
    assert not bad, bad[:5]


def test_config3_sized_pairs(gpu_ctx):
    """3 kb consensus pairs (config 3): 2-8 % divergence, some with a 100-600 bp
    insertion, compared with the oracle; plus a size-independent property at
    full size: MisScore(x, x) == 0 and the counts are symmetric in length."""
    PC = _pc()
    rng = random.Random(23)
    pairs = []
    for k in range(40):
        a = "".join(rng.choice("ACGT") for _ in range(rng.randint(2500, 3500)))
        pairs.append((a, mutate(rng, a, rng.choice([0.02, 0.05, 0.08]), ins=rng.choice([0, 0, 100, 600]))))
    st = []
    got = PC.aligment_score_batch(pairs, context=gpu_ctx, stats=st)
    exp = [P2.AligmentScore_c(a, b) for a, b in pairs]
    assert got == exp
    s = st[0][1]
    assert s["pairs"] == len(pairs) and s["dp_cells"] == sum(len(a) * len(b) for a, b in pairs)
    same = PC.aligment_score_batch([(a, a) for a, _ in pairs[:8]], context=gpu_ctx)
    assert same == [0] * 8


def test_calculate_misscore_and_pipe(gpu_ctx, tmp_path):
    PC = _pc()
    rng = random.Random(24)
    rows, lines = [], []
    for w in range(30):
        base = "".join(rng.choice("ACGT") for _ in range(rng.randint(200, 900)))
        som = ";".join(mutate(rng, base, 0.05, ins=rng.choice([0, 60])) for _ in range(rng.randint(1, 3)))
        ger = ";".join(mutate(rng, base, 0.05) for _ in range(rng.randint(1, 3)))
        flag = "NormalOutput|EMOutput" if w % 4 else "NormalOutput"
        r = ["chr1", 1000 * w, 1000 * w + 900, som, "a_tumor,b_tumor", "2", ger, "c_normal", "1", flag]
        rows.append(r)
        lines.append("\t".join(map(str, r)))
    f = tmp_path / "t.Raw.bed"
    f.write_text("\n".join(lines) + "\n")
    res = PC.MisScorePipe(str(f), context=gpu_ctx)
    exp = [P2.CalculateMisscore({"somSeqList": r[3], "germSeqList": r[6]}, score_fn=P2.AligmentScore_c)
           for r in rows if r[9] == "NormalOutput|EMOutput"]
    assert list(res["MisScore"]) == exp
    one = [r for r in rows if r[9] == "NormalOutput|EMOutput"][0]
    assert PC.CalculateMisscore({"somSeqList": one[3], "germSeqList": one[6]}) == exp[0]


def test_int32_fill_and_long_pairs(gpu_ctx, monkeypatch):
    """The int32 fill kernel (forced with SVS_MS_FILL=32, and taken by pairs
    longer than the packed kernel's 30000) gives the same counts; an odd
    number of packable pairs leaves one duo with a single pair."""
    PC = _pc()
    rng = random.Random(25)
    pairs = [random_pair(rng, max_len=200) for _ in range(501)]
    exp = [P2.AligmentScore_c(a, b) for a, b in pairs]
    assert PC.aligment_score_batch(pairs, context=gpu_ctx) == exp
    monkeypatch.setenv("SVS_MS_FILL", "32")
    assert PC.aligment_score_batch(pairs, context=gpu_ctx) == exp
    monkeypatch.delenv("SVS_MS_FILL")
    base = "".join(rng.choice("ACGT") for _ in range(150))
    long_pairs = [("".join(rng.choice("ACGT") for _ in range(31000)), base), (base, mutate(rng, base, 0.1)),
                  ("ACGT" * 7600, "ACGA" * 50)]
    assert PC.aligment_score_batch(long_pairs, context=gpu_ctx) == [P2.AligmentScore_c(a, b) for a, b in long_pairs]


def test_misscore_on_local_graph_output(gpu_ctx, tmp_path):
    """AlnFeature's MisScore over a Raw.bed that this build's localGraph wrote
    (synthetic windows with somatic insertions): MisScorePipe on the GPU equals
    the oracle's CalculateMisscore over the same records."""
    PC = _pc()
    from svscope_amd import synth
    from svscope_amd.local_graph import record_line
    from svscope_amd.som_td_detector import TDscope_npz_batch
    rows = [synth.make_window(w, 16, 700) for w in range(24)]
    recs = TDscope_npz_batch(rows, context=gpu_ctx)
    f = tmp_path / "T.vs.N.TandemRepeat.Raw.bed"
    f.write_text("\n".join(record_line(r) for r in recs) + "\n")
    em = [r for r in recs if str(r[-1]) == "NormalOutput|EMOutput"]
    assert em, "no EMOutput window in the sample"
    res = PC.MisScorePipe(str(f), context=gpu_ctx)
    exp = [P2.CalculateMisscore({"somSeqList": str(r[3]), "germSeqList": str(r[6])}, score_fn=P2.AligmentScore_c)
           for r in em]
    assert list(res["MisScore"]) == exp


def test_traceback_variants_agree(gpu_ctx, monkeypatch):
    """The wave-per-pair tiled traceback (default) and the lane-per-pair one
    (SVS_MS_TB=lane) give the oracle's counts, cutoffs included."""
    PC = _pc()
    rng = random.Random(26)
    pairs = [random_pair(rng, max_len=120) for _ in range(600)]
    for _ in range(6):
        a = "".join(rng.choice("ACGT") for _ in range(3000))
        pairs.append((a, mutate(rng, a, 0.08, ins=rng.choice([0, 500]))))
    for cut in (0, 5):
        exp = [P2.AligmentScore_c(a, b, cut) for a, b in pairs]
        assert PC.aligment_score_batch(pairs, cutoff=cut, context=gpu_ctx) == exp
        monkeypatch.setenv("SVS_MS_TB", "lane")
        assert PC.aligment_score_batch(pairs, cutoff=cut, context=gpu_ctx) == exp
        monkeypatch.delenv("SVS_MS_TB")


def test_unsupported_cutoff_fails_loudly(gpu_ctx):
    """cutoff > 64 is outside the kernel's flag window: an error, never a
    silently different count (the reference only calls cutoff=0)."""
    from svscope_amd import _abi
    PC = _pc()
    with pytest.raises(_abi.SvsError):
        PC.AligmentScore("ACGT" * 50, "ACGA" * 50, cutoff=65)


def test_misscore_on_config3_local_graph_output(gpu_ctx, tmp_path):
    """Full size: the consensus pairs of 8 config-3 windows (64 reads x 3 kb)
    written by this build's localGraph, through MisScorePipe on the GPU,
    equal the oracle's CalculateMisscore."""
    PC = _pc()
    from svscope_amd import synth
    from svscope_amd.local_graph import record_line
    from svscope_amd.som_td_detector import TDscope_npz_batch
    rows = [synth.make_window(w, 64, 3000) for w in range(200, 208)]
    recs = TDscope_npz_batch(rows, context=gpu_ctx)
    f = tmp_path / "T.vs.N.TandemRepeat.Raw.bed"
    f.write_text("\n".join(record_line(r) for r in recs) + "\n")
    em = [r for r in recs if str(r[-1]) == "NormalOutput|EMOutput"]
    assert em
    res = PC.MisScorePipe(str(f), context=gpu_ctx)
    exp = [P2.CalculateMisscore({"somSeqList": str(r[3]), "germSeqList": str(r[6])}, score_fn=P2.AligmentScore_c)
           for r in em]
    assert list(res["MisScore"]) == exp
