"""Decision oracle (literal restatement of DataScanner/DecisionMaker) pinned
against records the reference's own Decision produced (gen_decision_goldens.py)."""
import json
import os

import numpy as np

from oracle import decision_oracle

GOLD = os.path.join(os.path.dirname(__file__), "golden", "decision_goldens.json")


def test_decision_oracle_matches_reference_records():
    cases = json.load(open(GOLD))
    assert len(cases) >= 12
    for c in cases:
        rec = decision_oracle.tdscope_npz(c["TDRecord"], c["sequenceList"], np.array(c["ReadIDs"]),
                                          c["flank_5"], c["flank_3"])
        assert decision_oracle.record_line(rec) == c["line"], c["kind"]


def test_feature_selection_matches_reference():
    for c in json.load(open(GOLD)):
        if not c["features"]:
            continue
        enc, feat, rid = decision_oracle.msa_feature_selection(c["sequenceList"], c["flank_5"], c["flank_3"],
                                                               np.array(c["ReadIDs"]))
        assert list(enc.shape) == c["features"]["encoded_shape"]
        assert feat.tolist() == c["features"]["seqdatamx"]
        assert list(map(str, rid)) == c["features"]["read_ids"]


def test_goldens_cover_edge_cases():
    kinds = {c["kind"] for c in json.load(open(GOLD))}
    assert {"empty_read", "one_tag", "few_reads", "germline_only", "empty_flanks"} <= kinds
    lines = [c["line"] for c in json.load(open(GOLD))]
    assert any(l.endswith("|EMOutput") for l in lines)
