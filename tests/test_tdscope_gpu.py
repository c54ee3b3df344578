"""TDscope with its DUP corner re-scan (SomTDDetector.py:26-61) and the
BAM-reading localGraph (SVscope.py:118-183) on the GPU, against records the
reference's own TDscope wrote over the same synthetic BAM
(tests/golden/datamaker_goldens.json): the first Decision's EMOutput, the 5'
corner's (Record5), the 3' corner's (Record3) and the flag rewrite."""
import functools
import json
import os
from types import SimpleNamespace

import pytest

from svscope_amd import data_maker as dmk
from tests import fake_bam

pytestmark = pytest.mark.gpu

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "datamaker_goldens.json")))
READERS = fake_bam.FakeReaders()
REF, BAMS, LABELS = fake_bam.paths(GOLD["dataset"])


def _partials():
    kw = dict(refFile=REF, bamFileList=BAMS, LabelList=LABELS, offset=GOLD["offset"], mapQ=GOLD["mapQ"],
              readers=READERS)
    return functools.partial(dmk.DataMaker, **kw), functools.partial(dmk.DataMaker2, **kw)


def _line(rec):
    return "\t".join(str(x) for x in rec)


def test_tdscope_per_window_matches_reference():
    from svscope_amd.decision_maker import Decision
    from svscope_amd.som_td_detector import TDscope
    dm, dm2 = _partials()
    dec = functools.partial(Decision, Tlabel="tumor", readcutoff=3, hcutoff=3, scutoff=0.05)
    for c in GOLD["cases"]:
        assert _line(TDscope(c["TDRecord"], dm, dm2, dec)) == c["line"], c["TDRecord"]


def test_tdscope_batch_matches_reference():
    from svscope_amd.som_td_detector import TDscope_batch
    dm, dm2 = _partials()
    recs = TDscope_batch([c["TDRecord"] for c in GOLD["cases"]], dm, dm2)
    assert [_line(r) for r in recs] == [c["line"] for c in GOLD["cases"]]


def test_local_graph_bam_end_to_end(tmp_path):
    from svscope_amd.local_graph import localGraph, sort_lines
    bed = tmp_path / "win.bed"
    bed.write_text("".join(c["TDRecord"] + "\n" for c in GOLD["cases"]))
    args = SimpleNamespace(windowBed=str(bed), Tumorbam=BAMS[0], Normalbam=BAMS[1], TSampleID="T1",
                           NSampleID="N1", Reference=REF, savedir=str(tmp_path / "out"), thread="1",
                           offset=GOLD["offset"], mapQ=GOLD["mapQ"], Continue=False, batch=3)
    path = localGraph(args, readers=READERS)
    assert os.path.basename(path) == "T1.vs.N1.TandemRepeat.Raw.bed"
    got = open(path).read().splitlines()
    assert got == sort_lines([c["line"] for c in GOLD["cases"]])
