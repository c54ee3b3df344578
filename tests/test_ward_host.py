"""Host ward linkage + maxclust (svs_ward_maxclust_batch) vs the installed scipy.

The reference initialises EM with scipy's linkage(S, 'ward') and
fcluster(Z, K, 'maxclust') (ReadsCluster.py:243, :94).  The engine restates
both in C++ (svscope_amd/csrc/ward.cpp); labels must be identical to scipy's
for every K, including on tied and degenerate similarity matrices.
"""
import ctypes
import warnings

import numpy as np
import pytest
from scipy.cluster.hierarchy import ClusterWarning, fcluster, linkage

from svscope_amd import _abi


def scipy_labels(S, kmax):
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", ClusterWarning)
        Z = linkage(S, "ward")
    return np.stack([fcluster(Z, K, criterion="maxclust") for K in range(1, kmax)]).astype(np.int32)


def engine_labels(mats, max_c=9):
    lib = _abi.load_library()
    wins = (_abi.EmWindow * len(mats))()
    s_off = np.zeros(len(mats), np.int64)
    blobs, lab_off, tot_s, tot_l = [], [], 0, 0
    for w, S in enumerate(mats):
        n = S.shape[0]
        wins[w].n_reads = n
        wins[w].n_feat = 1
        wins[w].label_off = tot_l
        s_off[w] = tot_s
        blobs.append(np.ascontiguousarray(S, np.float64).reshape(-1))
        tot_s += n * n
        tot_l += (min(max_c + 1, n) - 1) * n
    S_blob = np.concatenate(blobs)
    labels = np.full(max(1, tot_l), -7, np.int32)
    _abi.check(lib.svs_ward_maxclust_batch(len(mats), wins, S_blob.ctypes.data_as(ctypes.c_void_p),
                                           s_off.ctypes.data_as(ctypes.c_void_p), max_c,
                                           labels.ctypes.data_as(ctypes.c_void_p)), "svs_ward_maxclust_batch")
    out = []
    for w, S in enumerate(mats):
        n = S.shape[0]
        k = min(max_c + 1, n) - 1
        out.append(labels[wins[w].label_off:wins[w].label_off + k * n].reshape(k, n))
    return out


def _cases():
    rng = np.random.default_rng(11)
    cases = []
    for n in (3, 4, 5, 7, 10, 16, 33, 64):
        for _ in range(6):
            cases.append(rng.random((n, n)))                                # generic reals
            cases.append(rng.integers(0, 3, (n, n)).astype(np.float64))     # heavy ties
            X = rng.integers(0, 5, (n, 20))                                 # similarity-like
            cases.append((X[:, None, :] == X[None, :, :]).mean(-1))
    for n in (3, 6, 64):
        cases.append(np.zeros((n, n)))                                      # all distances 0
        base = rng.random(n)
        cases.append(np.tile(base, (n, 1)))                                 # identical rows
        M = rng.random((n, n))
        M[n // 2:] = M[0]                                                    # duplicate block
        cases.append(M)
    return cases


def test_ward_maxclust_matches_scipy():
    cases = _cases()
    got = engine_labels(cases)
    for S, g in zip(cases, got):
        exp = scipy_labels(S, min(10, S.shape[0]))
        np.testing.assert_array_equal(g, exp, err_msg=f"n={S.shape[0]}")


def test_ward_maxclust_em_like_windows():
    """Similarity matrices of the kind EMCluster builds (pariwiseDistance of 0..4 symbols)."""
    from oracle.em_oracle import similarity
    rng = np.random.default_rng(5)
    mats = []
    for _ in range(40):
        n = int(rng.integers(6, 65))
        nf = int(rng.integers(10, 60))
        hap = rng.integers(0, 5, (3, nf))
        X = hap[rng.integers(0, 3, n)].copy()
        noise = rng.random(X.shape) < 0.1
        X[noise] = rng.integers(0, 5, noise.sum())
        mats.append(similarity(X.astype(np.uint8)))
    got = engine_labels(mats)
    for S, g in zip(mats, got):
        np.testing.assert_array_equal(g, scipy_labels(S, min(10, S.shape[0])))


def test_ward_maxclust_rejects_bad_args():
    lib = _abi.load_library()
    assert lib.svs_ward_maxclust_batch(1, None, None, None, 9, None) == -1
    wins = (_abi.EmWindow * 1)()
    S = np.zeros(4)
    off = np.zeros(1, np.int64)
    lab = np.zeros(4, np.int32)
    wins[0].n_reads = 0
    assert lib.svs_ward_maxclust_batch(1, wins, S.ctypes.data_as(ctypes.c_void_p),
                                       off.ctypes.data_as(ctypes.c_void_p), 9,
                                       lab.ctypes.data_as(ctypes.c_void_p)) == -1


@pytest.mark.parametrize("n", [3, 64])
def test_ward_maxclust_random_sweep(n):
    rng = np.random.default_rng(100 + n)
    mats = [rng.random((n, n)).round(int(rng.integers(1, 4))) for _ in range(200)]
    got = engine_labels(mats)
    for S, g in zip(mats, got):
        np.testing.assert_array_equal(g, scipy_labels(S, min(10, n)))
