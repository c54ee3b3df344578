"""Window extraction (svscope_amd/data_maker.py) against the reference's own
DataScanner / SomTDDetector_AimDatFetch code run over the same synthetic BAM
(tests/golden/datamaker_goldens.json, gen_datamaker_goldens.py), and the
.npz bundle writer read back by localGraph_npz's loader.  CPU only."""
import functools
import json
import os

import numpy as np
import pytest

from svscope_amd import data_maker as dmk
from tests import fake_bam

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "datamaker_goldens.json")))
READERS = fake_bam.FakeReaders()
REF, BAMS, LABELS = fake_bam.paths(GOLD["dataset"])
OFF, MAPQ = GOLD["offset"], GOLD["mapQ"]


def _plain(x):
    if isinstance(x, np.ndarray):
        return {"ndarray": [str(v) for v in x.tolist()]}
    if isinstance(x, (list, tuple)):
        return [_plain(v) for v in x]
    if isinstance(x, np.integer):
        return int(x)
    return x


def test_dataset_matches_golden_windows():
    assert [c["TDRecord"] for c in GOLD["cases"]] == fake_bam.dataset(GOLD["dataset"])[2]


@pytest.mark.parametrize("k", range(len(GOLD["cases"])))
def test_extractors_match_reference(k):
    c = GOLD["cases"][k]
    w = c["TDRecord"]
    assert _plain(dmk.FetchTDsubSeq(REF, BAMS, LABELS, w, offset=OFF, readers=READERS)) == c["FetchTDsubSeq"]
    assert _plain(dmk.DataMaker(w, REF, BAMS, LABELS, offset=OFF, mapQ=MAPQ, readers=READERS)) == c["DataMaker"]
    assert _plain(dmk.DataMaker2(w, REF, BAMS, LABELS, offset=OFF, mapQ=MAPQ, readers=READERS)) == c["DataMaker2"]
    chrom, start, end = w.split("\t")[0:3]
    corner = "\t".join([chrom, start, str(int(start) + 50)])
    assert _plain(dmk.SubSeqInWindow(BAMS, LABELS, corner, readers=READERS)) == c["SubSeqInWindow"]
    row = dmk.BundleMaker(w, REF, BAMS, LABELS, offset=OFF, mapQ=MAPQ, readers=READERS)
    assert row.dtype == object and row.shape == (5,)
    assert _plain(list(row)) == c["bundle_row"]


def test_every_extraction_branch_is_covered():
    flags = [c["DataMaker"][5] for c in GOLD["cases"]]
    assert {"NormalOutput", "GapRegion", "NoEnoughspanReads"} <= set(flags)
    outcomes = [c["TDscope"][-1] for c in GOLD["cases"]]
    assert "UnspanedSV|EMOutput" in outcomes and "UnspannedSV|EMOutput" in outcomes  # Record5, Record3
    assert "UnspanedSV" in outcomes  # flag rewrite
    assert outcomes.count("NormalOutput|EMOutput") >= 2  # first call, incl. a DUP window


def test_partials_pickle():
    import pickle
    dm = functools.partial(dmk.DataMaker, refFile=REF, bamFileList=BAMS, LabelList=LABELS, offset=OFF, mapQ=MAPQ,
                           readers=READERS)
    dm2 = pickle.loads(pickle.dumps(dm))
    w = GOLD["cases"][0]["TDRecord"]
    assert _plain(dm2(w)) == GOLD["cases"][0]["DataMaker"]


def test_missing_pysam_fails_loudly():
    try:
        import pysam  # noqa: F401
        pytest.skip("pysam is installed")
    except ImportError:
        pass
    with pytest.raises(ImportError):
        dmk.DataMaker(GOLD["cases"][0]["TDRecord"], "ref.fa", ["t.bam"], ["T1_tumor"])


def test_bundle_writer_round_trip(tmp_path):
    """save_bundles (SomTDDetector_AimDatFetch.py:160-183) -> the .npz files
    localGraph_npz loads (SVscope.py:209-212): same rows, block split, names."""
    from svscope_amd.local_graph import load_bundles, _window
    rows = [dmk.BundleMaker(c["TDRecord"], REF, BAMS, LABELS, offset=OFF, mapQ=MAPQ, readers=READERS)
            for c in GOLD["cases"]]
    paths = dmk.save_bundles(rows, str(tmp_path), ["T1"], ["N1"], block=3)
    assert [os.path.basename(p) for p in paths] == ["T1.vs.N1.TandemRepeat.batch%d.npz" % b for b in range(3)]
    dat = np.load(paths[0], allow_pickle=True)["DatSet"]  # our own file
    assert dat.shape == (3, 5) and dat.dtype == object
    back = load_bundles(str(tmp_path))
    assert len(back) == len(rows)
    for got, exp, c in zip(back, rows, GOLD["cases"]):
        assert _plain(list(got)) == _plain(list(exp)) == c["bundle_row"]
        rec, seqs, ids, f5, f3 = _window(got)
        assert rec == c["TDRecord"] and list(seqs) == list(exp[0]) and list(ids) == list(exp[1])


def _oracle_decision_batch(windows, **kw):
    from oracle import decision_oracle
    out = []
    for w in windows:
        np.random.seed(2023)
        rec, seqs, ids, f5, f3 = w[:5]
        out.append(decision_oracle.decision(rec, list(seqs), np.asarray(ids), f5, f3,
                                            window_flag=w[5] if len(w) > 5 else "NormalOutput"))
    return out


def test_local_graph_bam_plumbing_with_oracle_decisions(tmp_path, monkeypatch):
    """localGraph's host side (spawned extraction pool, chunking, DUP re-scan
    batching, journal, sort) with the CPU oracle standing in for the GPU
    DecisionBatch: the reference TDscope's records, sorted."""
    from types import SimpleNamespace
    from svscope_amd import local_graph, som_td_detector
    monkeypatch.setattr(som_td_detector, "DecisionBatch", _oracle_decision_batch)
    bed = tmp_path / "win.bed"
    bed.write_text("".join(c["TDRecord"] + "\n" for c in GOLD["cases"]))
    args = SimpleNamespace(windowBed=str(bed), Tumorbam=BAMS[0], Normalbam=BAMS[1], TSampleID="T1",
                           NSampleID="N1", Reference=REF, savedir=str(tmp_path / "out"), thread="2",
                           offset=OFF, mapQ=MAPQ, Continue=False, batch=3)
    path = local_graph.localGraph(args, readers=READERS)
    exp = local_graph.sort_lines([c["line"] for c in GOLD["cases"]])
    assert open(path).read().splitlines() == exp
    # --Continue with everything written: nothing re-run, same file
    args.Continue = True
    monkeypatch.setattr(som_td_detector, "DecisionBatch", lambda *a, **k: pytest.fail("re-ran a finished window"))
    local_graph.localGraph(args, readers=READERS)
    assert open(path).read().splitlines() == exp


class _ListReaders:
    """readers hook over explicit read lists (one per BAM path)."""

    def __init__(self, bams):
        self.bams = bams

    def alignment(self, path):
        reads = self.bams[path]

        class _F:
            def fetch(self, contig, start=None, stop=None):
                return [r for r in reads if r.reference_start < stop and r.reference_end > start]
        return _F()


def _linear_read(name, start, length, rs, secondary=False):
    seq = "".join(rs.choice(list("ACGT"), length))
    pairs = [(i, start + i) for i in range(length)]
    return fake_bam.FakeRead(name, seq, 60, start, pairs, [(0, length)], secondary=secondary)


def test_duplicate_primary_names_fail_only_when_spanning():
    """DataScanner.py:113-117: SeqDf.loc[spanReadIDs] + the axis-1 concat fail
    only when a span name has two primary rows; a duplicated primary name that
    does not span both flanks is ignored."""
    rs = np.random.RandomState(7)
    rec = "chrF\t1000\t1100\tX\t0"
    span = [_linear_read("s%d" % i, 700, 700, rs) for i in range(4)]
    # a name with two primaries, neither spanning both flanks (F5 = 800..1000, F3 = 1100..1300)
    dup = [_linear_read("d", 900, 300, rs), _linear_read("d", 1050, 200, rs)]
    base = dmk.FetchTDsubSeq("ref", ["b0"], ["T1_tumor"], rec, offset=200,
                             readers=_ListReaders({"b0": span}))
    got = dmk.FetchTDsubSeq("ref", ["b0"], ["T1_tumor"], rec, offset=200,
                            readers=_ListReaders({"b0": span + dup}))
    assert got == base and len(got[0]) == 4
    # one primary spans F5 only, the other F3 only: "d" is a span name with two
    # primary rows -> the reference's concat raises
    a, b = _linear_read("d", 700, 320, rs), _linear_read("d", 1080, 250, rs)
    with pytest.raises(ValueError):
        dmk.FetchTDsubSeq("ref", ["b0"], ["T1_tumor"], rec, offset=200, readers=_ListReaders({"b0": span + [a, b]}))
