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


@pytest.fixture(scope="module", params=["rows", "strip", "strip-pruned"])
def emu(request):
    """The emulator in both table layouts: row-major tables (export_rows)
    and the strip-major planner with register pass-through (poa_strip.hip);
    "strip-pruned" also re-runs every alignment with the exact pruning at its
    tightest bound (lb = the optimum: same alignment required) and just above
    it (a retry required)."""
    lib = helpers.build_emu()
    os.environ.pop("EMU_PRUNE", None)
    if request.param.startswith("strip"):
        os.environ["EMU_STRIP"] = "1"
    else:
        os.environ.pop("EMU_STRIP", None)
    if request.param == "strip-pruned":
        os.environ["EMU_PRUNE"] = "1"
    yield lib
    os.environ.pop("EMU_STRIP", None)
    os.environ.pop("EMU_PRUNE", None)


def test_emulator_matches_oracle_random(emu):
    for seqs in helpers.random_cases(11, 250):
        assert helpers.emu_poa(emu, seqs) == oracle_poa(seqs, 1), seqs


def test_emulator_matches_oracle_synthetic_windows(emu):
    from svscope_amd import synth
    for w in range(3):
        win = synth.make_window(w, 8, 500)
        assert helpers.emu_poa(emu, win[0]) == oracle_poa(win[0], 1)


def test_emulator_pruning_skips_rows():
    """At the tightest bound the pruning leaves most strip rows of a window
    MSA uncomputed (and the alignments unchanged, checked inside emu_poa)."""
    import ctypes
    from svscope_amd import synth
    lib = helpers.build_emu()
    lib.emu_prune_rows.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]
    os.environ["EMU_STRIP"] = "1"
    os.environ["EMU_PRUNE"] = "1"
    try:
        seqs = synth.make_window(4, 8, 1500)[0]
        enc = [x.encode() for x in seqs]
        h = lib.emu_poa(len(enc), (ctypes.c_char_p * len(enc))(*enc),
                        (ctypes.c_int * len(enc))(*[len(x) for x in enc]), 5, -4, -8, -6, -10, -4)
        try:
            assert lib.emu_error(h) is None, lib.emu_error(h)
            out = (ctypes.c_uint64 * 3)()
            lib.emu_prune_rows(h, out)
            assert 0 < out[0] < 0.6 * out[1], list(out)
        finally:
            lib.emu_free(h)
    finally:
        os.environ.pop("EMU_STRIP", None)
        os.environ.pop("EMU_PRUNE", None)
