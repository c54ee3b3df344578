"""Host-side MSA encoding / flank margin / feature selection of the product
(vectorised) against the oracle's literal restatement of DataScanner.py."""
import random

import numpy as np
import pytest

from oracle import decision_oracle as O
from svscope_amd import data_scanner as D


def rand_msa(rnd, rows, cols, gap=0.3):
    return ["".join("-" if rnd.random() < gap else rnd.choice("ATCG") for _ in range(cols)) for _ in range(rows)]


def test_encoder_decoder_roundtrip():
    assert D.SeqEncoder("AtCg-").tolist() == [0, 1, 2, 3, 4]
    assert O.seq_encoder("AtCg-").tolist() == [0, 1, 2, 3, 4]
    with pytest.raises(KeyError):
        D.SeqEncoder("ACGN")
    assert D.SeqDecoder(np.array([0, 4, 1, 2, 4, 3])) == "ATCG" == O.seq_decoder([0, 4, 1, 2, 4, 3])
    assert D.SeqDecoder(np.array([4, 4])) == ""


def test_call_margin_matches_literal_walk():
    rnd = random.Random(3)
    for t in range(600):
        cols = rnd.randint(1, 40)
        msa = rand_msa(rnd, 1, cols, gap=rnd.choice([0.0, 0.2, 0.6]))
        ung = msa[0].replace("-", "")
        k5, k3 = rnd.randint(0, 6), rnd.randint(0, 6)
        choice = rnd.random()
        f5 = ung[:k5] if choice < 0.6 else "".join(rnd.choice("ATCG") for _ in range(k5))
        tail = msa[0][1:].replace("-", "")
        f3 = (tail[-k3:] if k3 else "") if rnd.random() < 0.6 else "".join(rnd.choice("ATCG") for _ in range(k3))
        a = np.sort(np.unique(D.CallMargin(msa, f5, f3).astype(int)))
        b = np.sort(np.unique(O.call_margin(msa, f5, f3).astype(int)))
        assert a.tolist() == b.tolist(), (msa, f5, f3)


def test_find_non_same_site_matches():
    rs = np.random.RandomState(0)
    for _ in range(50):
        M = rs.randint(0, 5, size=(rs.randint(1, 30), rs.randint(0, 50)))
        for cut in (1, 3, 4.5):
            assert D.FindNonSameSite(M, cut).tolist() == O.find_non_same_site(M, cut).tolist()
