"""AlnFeature end to end with MisScore on the GPU (svs_aligment_score_batch)
against the reference AlnFeature's outputs over the same synthetic workspace
(tests/golden/alnfeature_goldens.json): Somatic.bed, RandomForestResult.tsv,
the VCF and the merged VCF."""
import pytest

from tests.test_aln_feature_host import check_outputs, run_alnfeature

pytestmark = pytest.mark.gpu


def test_alnfeature_matches_reference_on_gpu(tmp_path):
    _, merged = run_alnfeature(tmp_path, thread="1")
    check_outputs(tmp_path, merged)
