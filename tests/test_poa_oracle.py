"""Oracle (CPU spoa restatement) against hand-derived fixtures, and the kernel
emulator (CPU restatement of the HIP kernel's wave algorithm + the product's
host graph engine) against the oracle."""
import json
import os

import pytest

from oracle.spoa_oracle import poa as oracle_poa
from tests import helpers

GOLD = os.path.join(os.path.dirname(__file__), "golden", "poa_handchecked.json")


def test_oracle_hand_checked_fixtures():
    cases = json.load(open(GOLD))
    assert len(cases) >= 8
    for case in cases:
        cons, msa = oracle_poa(case["seqs"], 1)
        assert cons == case["consensus"], case
        assert msa == case["msa"], case


def test_oracle_rejects_unsupported_modes():
    with pytest.raises(RuntimeError):
        oracle_poa(["ACGT", "ACGT"], 0)


@pytest.fixture(scope="module", params=["rows", "strip"])
def emu(request):
    """The emulator in both kernel layouts: row-major tables (poa_kernels.hip)
    and the strip-major planner with register pass-through (poa_strip.hip)."""
    lib = helpers.build_emu()
    if request.param == "strip":
        os.environ["EMU_STRIP"] = "1"
    else:
        os.environ.pop("EMU_STRIP", None)
    yield lib
    os.environ.pop("EMU_STRIP", None)


def test_emulator_matches_oracle_random(emu):
    for seqs in helpers.random_cases(11, 250):
        assert helpers.emu_poa(emu, seqs) == oracle_poa(seqs, 1), seqs


def test_emulator_matches_oracle_synthetic_windows(emu):
    from svscope_amd import synth
    for w in range(3):
        win = synth.make_window(w, 8, 500)
        assert helpers.emu_poa(emu, win[0]) == oracle_poa(win[0], 1)
