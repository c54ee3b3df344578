"""The CPU oracle against the reference's own decision code at the BASELINE
window sizes: tests/golden/reference_path_goldens.json
was produced by running /root/reference/src/DecisionMaker.Decision (and
ReadsCluster.EMCluster on the real seqdatamx of the config-3 windows) in this
container (gen_reference_path_goldens.py; spoa is the oracle POA, the rest is
the reference's code).  These tests tie the oracle digests that the GPU tests
and bench.py check against to the reference's records."""
import hashlib
import json
import os

import numpy as np
import pytest

from oracle import decision_oracle, em_oracle

GDIR = os.path.join(os.path.dirname(__file__), "golden")
REF = json.load(open(os.path.join(GDIR, "reference_path_goldens.json")))


def _windows(name):
    return [w for w in REF["windows"] if w["set"] == name]


def test_reference_goldens_cover_the_baseline_sizes():
    sets = REF["sets"]
    assert (sets["config3"]["reads"], sets["config3"]["ref_len"], len(_windows("config3"))) == (64, 3000, 16)
    assert (sets["config2"]["reads"], sets["config2"]["ref_len"], len(_windows("config2"))) == (32, 2000, 16)
    assert len(_windows("harsh")) == 4
    flags = [w["flag"] for w in REF["windows"]]
    assert sum(f.endswith("|EMOutput") for f in flags) >= 24 and "NormalOutput" in flags


@pytest.mark.parametrize("name", ["config3", "config2", "harsh"])
def test_reference_records_equal_oracle_digests(name):
    """Every reference record (as its digest) equals the committed oracle
    digest of the same window: the oracle digests of bench_config3_digests,
    config2_digests and harsh_digests are the reference's own records for
    these ids."""
    gold = json.load(open(os.path.join(GDIR, REF["sets"][name]["oracle_digests"])))
    for w in _windows(name):
        assert gold["digests"][w["window"]] == w["digest"], (name, w["window"])
        assert gold["flags"][w["window"]] == w["flag"], (name, w["window"])


def test_em_oracle_matches_reference_emcluster_at_config3_size():
    """em_oracle.em_cluster on the seqdatamx the reference's
    MSAFeatureSelection produced for 16 config-3 windows (64 reads, 1375-2052
    feature columns): K and labels exact, BICList within 1e-5
    (ReadsCluster.py:221-277)."""
    z = np.load(os.path.join(GDIR, "reference_em_inputs.npz"))
    n = 0
    for w in _windows("config3"):
        if "K" not in w:
            continue
        X = z[f"config3_{w['window']}"].astype(np.int64)
        assert X.shape == (w["n"], w["nf"])
        r = em_oracle.em_cluster(X)
        assert r["K"] == w["K"], w["window"]
        np.testing.assert_array_equal(r["Rclust"], w["Rclust"])
        np.testing.assert_allclose(r["BICList"], w["BICList"], rtol=1e-9, atol=1e-5)
        n += 1
    assert n == 16


def test_decision_oracle_reproduces_a_reference_config2_record():
    """The whole oracle window path (oracle POA, features, numpy EM, literal
    Decision) on one 32-read x 2 kb window writes the reference's record."""
    from svscope_amd import synth
    w = _windows("config2")[1]
    s = REF["sets"]["config2"]
    seqs, ids, f5, f3, rec = synth.make_window(w["window"], s["reads"], s["ref_len"])
    out = decision_oracle.tdscope_npz(rec, seqs, np.asarray(ids), f5, f3)
    assert hashlib.sha256(decision_oracle.record_line(out).encode()).hexdigest() == w["digest"]
