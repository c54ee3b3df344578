"""Host MSAFeatureSelection of the engine (svs_msa_features, csrc/features.cpp)
vs the reference's own outputs (tests/golden/decision_goldens.json) and the
literal oracle (oracle/decision_oracle.py, DataScanner.py:146-220).

The MSA both sides start from is the CPU POA oracle's, so these tests need no
GPU; the GPU decision tests cover the same code behind svs_decision_batch.
"""
import ctypes
import json
import os

import numpy as np
import pytest

from oracle import decision_oracle
from oracle.spoa_oracle import poa as oracle_poa
from svscope_amd import _abi

GOLD = os.path.join(os.path.dirname(__file__), "golden", "decision_goldens.json")


def engine_features(msa, f5, f3, seqs, n_ids, hcutoff=3, scutoff=0.05):
    lib = _abi.load_library()
    R = len(msa)
    W = len(msa[0]) if R else 0
    blob = "".join(msa).encode("latin-1") or b"\0"
    lens = np.array([len(s) for s in seqs[1:]], np.int32)
    if lens.size == 0:
        lens = np.zeros(1, np.int32)
    rows, nf, nmap = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
    cap = max(1, (R + n_ids) * max(W, 1))
    feat = np.zeros(cap, np.uint8)
    idm = np.zeros(max(1, 2 * n_ids), np.int32)
    b5, b3 = f5.encode("latin-1"), f3.encode("latin-1")
    _abi.check(lib.svs_msa_features(R, W, blob, b5, len(b5), b3, len(b3), len(seqs) - 1,
                                    lens.ctypes.data_as(ctypes.c_void_p), n_ids, hcutoff, scutoff,
                                    ctypes.byref(rows), ctypes.byref(nf), feat.ctypes.data_as(ctypes.c_void_p),
                                    cap, idm.ctypes.data_as(ctypes.c_void_p), ctypes.byref(nmap), idm.size),
               "svs_msa_features")
    return feat[:rows.value * nf.value].reshape(rows.value, nf.value), idm[:nmap.value]


def test_features_match_reference_goldens():
    n = 0
    for c in json.load(open(GOLD)):
        if not c["features"]:
            continue
        seqs = c["sequenceList"]
        _, msa = oracle_poa(seqs, 1)
        feat, idm = engine_features(msa, c["flank_5"], c["flank_3"], seqs, len(c["ReadIDs"]))
        assert feat.tolist() == c["features"]["seqdatamx"], c["kind"]
        assert [c["ReadIDs"][i] for i in idm] == c["features"]["read_ids"], c["kind"]
        n += 1
    assert n >= 5


def _random_window(rs, n_reads, L, n_empty=0, lower=False):
    ref = "".join(rs.choice(list("ACGT"), L))
    reads = []
    for _ in range(n_reads):
        s = list(ref)
        for _ in range(int(rs.randint(0, L // 10 + 1))):
            p = int(rs.randint(0, len(s)))
            op = rs.randint(0, 3)
            if op == 0:
                s[p] = rs.choice(list("ACGT"))
            elif op == 1:
                del s[p]
            else:
                s.insert(p, rs.choice(list("ACGT")))
        reads.append("".join(s))
    for k in rs.choice(n_reads, n_empty, replace=False):
        reads[k] = ""
    if lower:
        reads = [r.lower() if i % 3 == 0 else r for i, r in enumerate(reads)]
    ids = [f"S_{'tumor' if i % 2 else 'normal'}|r{i}" for i in range(n_reads)]
    return [ref] + reads, ids, ref


@pytest.mark.parametrize("seed", range(12))
def test_features_match_oracle_random(seed):
    rs = np.random.RandomState(seed)
    n_reads = int(rs.randint(4, 14))
    L = int(rs.randint(40, 160))
    n_empty = int(rs.randint(0, 3)) if seed % 3 == 0 else 0
    seqs, ids, ref = _random_window(rs, n_reads, L, n_empty, lower=seed % 4 == 1)
    flank_kind = seed % 4
    if flank_kind == 0:
        f5, f3 = ref[:10], ref[-10:]
    elif flank_kind == 1:
        f5, f3 = "", ""
    elif flank_kind == 2:
        f5, f3 = "ACGTACGTACGTACGT", ref[-5:]      # 5' flank that never matches
    else:
        f5, f3 = ref[:3], "TTTTTTTTTTTTTTTTTTTT"
    _, msa = oracle_poa(seqs, 1)
    feat, idm = engine_features(msa, f5, f3, seqs, len(ids), hcutoff=2, scutoff=0.05)
    enc, exp_feat, exp_ids = decision_oracle.msa_feature_selection(seqs, f5, f3, np.array(ids), hcutoff=2,
                                                                   scutoff=0.05)
    assert feat.shape == exp_feat.shape
    np.testing.assert_array_equal(feat, exp_feat)
    assert [ids[i] for i in idm] == list(map(str, exp_ids))


def test_features_reject_unknown_symbol():
    lib = _abi.load_library()
    msa = ["ACGN", "ACGT"]
    lens = np.array([4], np.int32)
    rows, nf, nmap = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
    buf = np.zeros(16, np.uint8)
    idm = np.zeros(4, np.int32)
    rc = lib.svs_msa_features(2, 4, "".join(msa).encode(), b"", 0, b"", 0, 1, lens.ctypes.data_as(ctypes.c_void_p),
                              1, 3, 0.05, ctypes.byref(rows), ctypes.byref(nf), buf.ctypes.data_as(ctypes.c_void_p),
                              16, idm.ctypes.data_as(ctypes.c_void_p), ctypes.byref(nmap), 4)
    assert rc == -1  # SVS_E_INVALID
    assert b"KeyError" in lib.svs_last_error()
