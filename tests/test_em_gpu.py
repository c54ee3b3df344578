"""GPU parity of the EM seam against the reference-generated goldens and the
numpy oracle: identical K and read->component labels, BIC and per-read
log-likelihoods within 1e-5 (north_star tolerance)."""
import numpy as np
import pytest

from oracle import em_oracle

pytestmark = pytest.mark.gpu

import os
GOLD = os.path.join(os.path.dirname(__file__), "golden", "em_goldens.npz")


def test_similarity_matches_oracle():
    from svscope_amd.reads_cluster import similarity_batch
    rs = np.random.RandomState(1)
    mats = [rs.randint(0, 5, size=(n, nf)) for n, nf in [(6, 10), (16, 200), (64, 1000), (5, 0)]]
    for X, S in zip(mats, similarity_batch(mats)):
        np.testing.assert_array_equal(S, em_oracle.similarity(X))


@pytest.fixture(params=["parallel", "in_order"])
def em_mode(request, monkeypatch):
    """Both EM kernel forms: the K-parallel speculation (default, with the
    in-order rerun of the windows it cannot place) and SVS_EM_SEQ=1, the
    in-order form for every window (em_kernels.hip)."""
    if request.param == "in_order":
        monkeypatch.setenv("SVS_EM_SEQ", "1")
    else:
        monkeypatch.delenv("SVS_EM_SEQ", raising=False)
    return request.param


def test_em_matches_reference_goldens(em_mode):
    from svscope_amd.reads_cluster import em_cluster_batch
    gold = np.load(GOLD)
    n = int(gold["n_cases"])
    mats = [gold[f"c{c:02d}_X"].astype(np.int64) for c in range(n)]
    got = em_cluster_batch(mats, want_params=True)
    for c, r in enumerate(got):
        p = f"c{c:02d}_"
        assert r["K"] == int(gold[p + "K"]), c
        np.testing.assert_array_equal(r["Rclust"], gold[p + "Rclust"])
        np.testing.assert_allclose(r["BICList"], gold[p + "BICList"], rtol=1e-9, atol=1e-5)
        np.testing.assert_allclose(r["lik"], gold[p + "lik"], rtol=0, atol=1e-5)
        np.testing.assert_allclose(r["gamma"], gold[p + "gamma"], rtol=0, atol=1e-7)
        np.testing.assert_allclose(r["pi"], gold[p + "pi"], rtol=0, atol=1e-9)
        np.testing.assert_allclose(r["theta"].sum(axis=(1, 2)), gold[p + "theta_sum"], rtol=1e-9)


def test_em_matches_reference_emcluster_at_config3_size(em_mode):
    """the GPU EM on the seqdatamx the reference's own
    MSAFeatureSelection produced for 16 config-3 windows (64 reads,
    1375-2052 features) gives the reference EMCluster's K and labels exactly
    and its BICList within 1e-5 (reference_path_goldens.json,
    gen_reference_path_goldens.py; ReadsCluster.py:221-277)."""
    import json
    from svscope_amd.reads_cluster import em_cluster_batch
    gdir = os.path.dirname(GOLD)
    ref = json.load(open(os.path.join(gdir, "reference_path_goldens.json")))
    z = np.load(os.path.join(gdir, "reference_em_inputs.npz"))
    wins = [w for w in ref["windows"] if w["set"] == "config3" and "K" in w]
    assert len(wins) == 16
    got = em_cluster_batch([z[f"config3_{w['window']}"].astype(np.int64) for w in wins])
    for w, r in zip(wins, got):
        assert r["K"] == w["K"], w["window"]
        np.testing.assert_array_equal(r["Rclust"], w["Rclust"])
        np.testing.assert_allclose(r["BICList"], w["BICList"], rtol=1e-9, atol=1e-5)


def test_em_matches_oracle_random_and_reinit_heavy(em_mode):
    """Random and re-initialisation-heavy windows against the oracle.  Four
    of them re-initialise at two or more K values (windows 0, 8, 9 and 12),
    which the K-parallel speculation cannot place (ReadsCluster.py:179-187:
    each K's dirichlet draws continue the stream the smaller K left), so the
    default mode must rerun them in order."""
    from svscope_amd.reads_cluster import em_cluster_batch
    rs = np.random.RandomState(42)
    mats = []
    for k in range(24):
        n = int(rs.choice([6, 9, 16, 33, 64]))
        nf = int(rs.choice([10, 37, 150, 600]))
        protos = rs.randint(0, 5, size=(3, nf))
        X = protos[rs.randint(0, 3, size=n)]
        flip = rs.random_sample(X.shape) < 0.1
        X[flip] = rs.randint(0, 5, size=int(flip.sum()))
        if k % 3 == 0:
            X[n // 2:] = X[0]  # duplicates force dirichlet re-initialisation
        mats.append(X)
    timing = {}
    got = em_cluster_batch(mats, want_params=True, timing=timing)
    if em_mode == "parallel":
        assert timing["em_reruns"] >= 4, timing
    else:
        assert timing["em_reruns"] == 0, timing
    for X, r in zip(mats, got):
        o = em_oracle.em_cluster(X)
        assert r["K"] == o["K"]
        np.testing.assert_array_equal(r["Rclust"], o["Rclust"])
        np.testing.assert_allclose(r["BICList"], o["BICList"], rtol=1e-9, atol=1e-5)
        np.testing.assert_allclose(r["lik"], o["lik"], rtol=0, atol=1e-5)


def test_emcluster_signature():
    from svscope_amd.reads_cluster import EMCluster
    gold = np.load(GOLD)
    X = gold["c05_X"].astype(np.int64)
    K, Xo, R, theta, gamma, pie, bics = EMCluster(X, initselection=1)
    assert K == int(gold["c05_K"]) and Xo is X
    assert theta.shape == (K, X.shape[1], 5) and gamma.shape == (X.shape[0], K) and pie.shape == (K,)


def test_em_matches_oracle_many_reads_and_wide_windows():
    """Windows beyond one 64-read chunk (up to the kernel's 256 reads) and a
    config-3-sized feature matrix (64 reads x ~1600 columns)."""
    from svscope_amd.reads_cluster import em_cluster_batch
    rs = np.random.RandomState(7)
    mats = []
    for n, nf in [(65, 40), (100, 80), (200, 30), (256, 24), (64, 1600)]:
        protos = rs.randint(0, 5, size=(2, nf))
        X = protos[rs.randint(0, 2, size=n)]
        flip = rs.random_sample(X.shape) < 0.08
        X[flip] = rs.randint(0, 5, size=int(flip.sum()))
        mats.append(X)
    got = em_cluster_batch(mats)
    for X, r in zip(mats, got):
        o = em_oracle.em_cluster(X)
        assert r["K"] == o["K"]
        np.testing.assert_array_equal(r["Rclust"], o["Rclust"])
        np.testing.assert_allclose(r["BICList"], o["BICList"], rtol=1e-9, atol=1e-5)
        np.testing.assert_allclose(r["lik"], o["lik"], rtol=0, atol=1e-5)


@pytest.fixture
def em_mfma(monkeypatch):
    monkeypatch.setenv("SVS_EM_MFMA", "1")


def test_em_mfma_variant_matches_reference_goldens(em_mfma):
    """The v_mfma_f64_16x16x4_f64 E-step contraction (SVS_EM_MFMA=1) keeps the
    reference's K and labels exactly, BIC / log-likelihood within 1e-5."""
    test_em_matches_reference_goldens("parallel")


def test_em_mfma_variant_matches_oracle(em_mfma):
    test_em_matches_oracle_random_and_reinit_heavy("parallel")
