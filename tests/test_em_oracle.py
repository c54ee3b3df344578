"""EM oracle (numpy restatement of ReadsCluster.EMCluster) pinned against the
golden vectors the reference itself produced (tests/golden/gen_em_goldens.py)."""
import os

import numpy as np
import pytest

from oracle import em_oracle

GOLD = os.path.join(os.path.dirname(__file__), "golden", "em_goldens.npz")


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD)  # allow_pickle=False


def cases(gold):
    return range(int(gold["n_cases"]))


def test_rng_stream_is_numpy_legacy(gold):
    e = np.random.RandomState(2023).standard_exponential(4096)
    np.testing.assert_array_equal(e, gold["rng_2023_exp"])
    d = np.random.RandomState(2023).dirichlet(np.ones(5), size=4)
    ex = gold["rng_2023_exp"][:20].reshape(4, 5)
    acc = (((ex[:, 0] + ex[:, 1]) + ex[:, 2]) + ex[:, 3]) + ex[:, 4]
    np.testing.assert_array_equal(d, ex * (1.0 / acc)[:, None])


def test_oracle_matches_reference_goldens(gold):
    for c in cases(gold):
        p = f"c{c:02d}_"
        X = gold[p + "X"].astype(np.int64)
        r = em_oracle.em_cluster(X)
        assert r["K"] == int(gold[p + "K"]), c
        np.testing.assert_array_equal(r["Rclust"], gold[p + "Rclust"])
        np.testing.assert_allclose(r["BICList"], gold[p + "BICList"], rtol=1e-9, atol=1e-6)
        np.testing.assert_allclose(r["lik"], gold[p + "lik"], rtol=0, atol=1e-5)
        np.testing.assert_allclose(r["gamma"], gold[p + "gamma"], rtol=0, atol=1e-9)
        np.testing.assert_allclose(r["pi"], gold[p + "pi"], rtol=0, atol=1e-12)
        if p + "theta" in gold:
            np.testing.assert_allclose(r["theta"], gold[p + "theta"], rtol=0, atol=1e-12)


def test_goldens_exercise_reinit(gold):
    n = 0
    for c in cases(gold):
        n += em_oracle.em_cluster(gold[f"c{c:02d}_X"].astype(np.int64))["reinits"] > 0
    assert n >= 3
