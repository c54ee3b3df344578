"""AlnFeature's host tail (svscope_amd/aln_feature.py) against the reference's
own AlnFeature run over the same synthetic workspace
(tests/golden/alnfeature_goldens.json, gen_alnfeature_goldens.py): alignment
DB, background coverage/mapQ/chromosome-span, the random-forest feature table,
the VCF and the merged VCF.  MisScore here comes from the CPU oracle (the GPU
run is tests/test_aln_feature_gpu.py).  CPU only."""
import io
import json
import os
from types import SimpleNamespace

import numpy as np
import pandas as pd
import pytest

from svscope_amd import aln_feature as af
from tests import fake_tabix

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "alnfeature_goldens.json")))
READERS = fake_tabix.FakeTabixReaders()


def _no_date(text):
    """Drops ##fileDate and the workspace directory of ##reference (the
    golden was written in a temporary directory)."""
    out = []
    for x in text.splitlines(True):
        if x.startswith("##fileDate"):
            continue
        if x.startswith("##reference="):
            x = "##reference=" + os.path.basename(x[len("##reference="):])
        out.append(x)
    return "".join(out)


def _oracle_misscore_pipe(path, context=None, stats=None):
    from oracle import pairwise2_oracle as pw
    df = pd.read_csv(path, sep="\t", header=None)
    df.columns = ["chrom", "start", "end", "somSeqList", "somSupportReadID", "someventCount", "germSeqList",
                  "germSupportReadID", "germeventCount", "flag"]
    som = df.loc[df["flag"] == "NormalOutput|EMOutput"].copy()
    som["window"] = som["chrom"] + "_" + som["start"].astype("str") + "-" + som["end"].astype("str")
    som["MisScore"] = [pw.CalculateMisscore(r, score_fn=pw.AligmentScore_c) for _, r in som.iterrows()]
    som["AF"] = [pw.CallAlleleFreq(r["somSupportReadID"], r["germSupportReadID"]) for _, r in som.iterrows()]
    return som[["chrom", "start", "end", "window", "somSupportReadID", "germSupportReadID", "MisScore", "AF"]]


def run_alnfeature(tmp_path, monkeypatch=None, thread="2"):
    paths = fake_tabix.write(str(tmp_path))
    args = SimpleNamespace(savedir=str(tmp_path), TSampleID="T1", NSampleID="N1", Tumorbam="t.bam",
                           Normalbam="n.bam", thread=thread, **paths)
    merged = af.AlnFeature(args, model=fake_tabix.StubForest(), readers=READERS)
    return args, merged


def check_outputs(tmp_path, merged):
    d = str(tmp_path)
    for name in ("T1.Somatic.bed", "RandomForestResult.tsv"):
        assert open(os.path.join(d, name)).read() == GOLD[name], name
    assert _no_date(open(os.path.join(d, "T1.vcf")).read()) == _no_date(GOLD["T1.vcf"])
    assert _no_date(open(merged).read()) == _no_date(GOLD["T1.mergedSomatic.vcf"])


def test_alnfeature_matches_reference_with_oracle_misscore(tmp_path, monkeypatch):
    from svscope_amd import pairwise_compare
    monkeypatch.setattr(pairwise_compare, "MisScorePipe", _oracle_misscore_pipe)
    _, merged = run_alnfeature(tmp_path)
    check_outputs(tmp_path, merged)


def test_background_and_db_match_reference(tmp_path):
    fake_tabix.write(str(tmp_path))
    d = str(tmp_path)
    tbed, nbed = os.path.join(d, "T1.bed.gz"), os.path.join(d, "N1.bed.gz")
    db_t = af.makeupDB(tbed, os.path.join(d, "Tumor"), readers=READERS)
    db_n = af.makeupDB(nbed, os.path.join(d, "Normal"), readers=READERS)
    assert [list(x) for x in af.query_reads(db_t, "rd00003")] == GOLD["query_reads"]
    bg = af.background(os.path.join(d, "genome.windows.bed"), tbed, db_t, workthread=1, readers=READERS)
    assert json.loads(bg.to_json(orient="split")) == GOLD["background_T_genome"]
    sv = af.background(os.path.join(d, "T1.vs.N1.TandemRepeat.Raw.bed"), nbed, db_n, showchromSpan=True,
                       workthread=2, readers=READERS)
    assert json.loads(sv.to_json(orient="split")) == GOLD["background_N_raw"]


def test_ovlen_cases():
    for w, s, e, exp in GOLD["OVLEN"]:
        assert af.OVLEN(w, s, e) == exp


def test_sv_type_thresholds():
    assert [af.sv_type(x) for x in (50, 49, -49, -50, 0, 400, -400)] == ["INS", "MisAlign", "MisAlign", "DEL",
                                                                          "MisAlign", "INS", "DEL"]


def test_model_is_required():
    with pytest.raises(TypeError):
        af.AlnFeature(SimpleNamespace())  # the caller must pass the forest (no pickle is loaded here)
