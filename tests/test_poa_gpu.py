"""GPU parity of the POA seam: svscope_amd.poa (HIP kernel through the C ABI)
against the CPU oracle, bit-exact on consensus and every MSA row."""
import ctypes

import numpy as np
import pytest

from oracle.spoa_oracle import poa as oracle_poa
from tests import helpers

pytestmark = pytest.mark.gpu


def test_wave_primitives(gpu_ctx):
    rs = np.random.RandomState(3)
    n_waves = 64
    x = rs.randint(-10 ** 6, 10 ** 6, size=n_waves * 64).astype(np.int32)
    x[::7] = -(2 ** 30)
    scan = np.zeros_like(x)
    shift = np.zeros_like(x)
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    from svscope_amd import _abi
    _abi.check(gpu_ctx.lib.svs_wave_selftest(gpu_ctx.handle, p(x), p(scan), p(shift), n_waves))
    xr = x.reshape(n_waves, 64)
    np.testing.assert_array_equal(scan.reshape(n_waves, 64), np.maximum.accumulate(xr, axis=1))
    exp_shift = np.concatenate([np.full((n_waves, 1), -7, np.int32), xr[:, :-1]], axis=1)
    np.testing.assert_array_equal(shift.reshape(n_waves, 64), exp_shift)


def test_handchecked_fixtures_on_gpu():
    import json, os
    from svscope_amd.poa import poa
    cases = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "poa_handchecked.json")))
    for c in cases:
        assert poa(c["seqs"], 1) == (c["consensus"], c["msa"]), c


def test_random_cases_batched_match_oracle():
    from svscope_amd.poa import poa_batch
    cases = helpers.random_cases(101, 400)
    got = poa_batch(cases)
    for seqs, g in zip(cases, got):
        assert g == oracle_poa(seqs, 1), seqs


def test_longer_random_cases_match_oracle():
    from svscope_amd.poa import poa_batch
    cases = helpers.random_cases(7, 60, max_seqs=12, max_len=300, edits=25)
    got = poa_batch(cases)
    for seqs, g in zip(cases, got):
        assert g == oracle_poa(seqs, 1)


def test_single_equals_batch():
    from svscope_amd.poa import poa, poa_batch
    cases = helpers.random_cases(5, 20)
    batched = poa_batch(cases)
    for seqs, b in zip(cases, batched):
        assert poa(seqs, 1) == b


def test_synthetic_windows_match_oracle():
    from svscope_amd import synth
    from svscope_amd.poa import poa_batch
    wins = [synth.make_window(w, 16, 2000) for w in range(2)] + [synth.make_window(7, 8, 3000)]
    got = poa_batch([w[0] for w in wins])
    for w, g in zip(wins, got):
        assert g == oracle_poa(w[0], 1)


def test_unsupported_modes_raise():
    from svscope_amd import _abi
    from svscope_amd.poa import poa
    with pytest.raises(_abi.SvsError):
        poa(["ACGT", "ACGA"], 0)
    with pytest.raises(_abi.SvsError):
        poa(["ACGT", "ACGA"], 1, g=-2, e=-6)  # linear subtype
    with pytest.raises(_abi.SvsError):
        poa(["ACGT", "ACGA"], 1, m=5000)  # beyond the 24-bit pruning-bound multiplies


def test_genmsa_false_and_min_coverage():
    from svscope_amd.poa import poa
    seqs = ["ACGTTGCA", "ACGTGCA", "ACGATGCA", "TTACGTTGCA"]
    cons, msa = poa(seqs, 1, genmsa=False)
    assert msa == [] and cons == oracle_poa(seqs, 1)[0]
    assert poa(seqs, 1, min_coverage=3) == oracle_poa(seqs, 1, min_coverage=3)


@pytest.mark.parametrize("env", [
    {"SVS_POA_WPJ": "1"},
    {"SVS_POA_WPJ": "2"},
    {"SVS_POA_WPJ": "4"},
    {"SVS_POA_WPJ": "8"},
    {"SVS_POA_WPJ": "16"},
    {"SVS_POA_STRIP_GLOBAL_POOL": "1", "SVS_POA_WPJ": "1"},
    {"SVS_POA_STRIP_GLOBAL_POOL": "1", "SVS_POA_WPJ": "4"},
    {"SVS_POA_PRUNE": "0"},
    {"SVS_POA_PRUNE_SLACK": "0", "SVS_POA_WPJ": "1"},
    {"SVS_POA_PRUNE_SLACK": "0", "SVS_POA_WPJ": "8"},
    {"SVS_POA_PRUNE_SLACK": "-0.3", "SVS_POA_WPJ": "4"},
    {"SVS_POA_PRUNE_SLACK": "0", "SVS_POA_STRIP_GLOBAL_POOL": "1", "SVS_POA_WPJ": "2"},
    {"SVS_POA_PRUNE_SLACK": "-0.3", "SVS_POA_PRUNE_RETRY_SLACK": "none"},
    {"SVS_POA_PRUNE_SLACK": "-0.3", "SVS_POA_PRUNE_RETRY_SLACK": "-0.3", "SVS_POA_PRUNE_MAX_RETRIES": "100"},
    {"SVS_POA_VERIFY_GRAPH": "1"},
    {"SVS_POA_SYNC_CHECK": "1", "SVS_POA_WPJ": "4"},
    {"SVS_POA_VERIFY_GRAPH": "1", "SVS_POA_PRUNE_SLACK": "-0.3", "SVS_POA_WPJ": "2"},
    {"SVS_POA_VERIFY_GRAPH": "1", "SVS_POA_SORT_STACK": "64"},
    {"SVS_POA_HOST_GRAPH": "1"},
    {"SVS_POA_HOST_GRAPH": "1", "SVS_POA_VERIFY_PREP": "1"},
    {"SVS_POA_HOST_GRAPH": "1", "SVS_POA_VERIFY_PREP": "1", "SVS_POA_PRUNE_SLACK": "-0.3"},
])
def test_kernel_variants_match_oracle(env):
    """Every POA kernel instance the engine selects gives the oracle's result:
    1/2/4/8/16 pipelined waves per job, the
    pool in global memory, and the exact pruning off, at its tightest slack,
    and with a bound above the optimum (every pruned job retried: with the
    looser retry slack, unpruned, or twice, the second time unpruned; with
    the tables exported straight into the staging buffer a retried job's
    block is exported again); with the device-resident graphs (the default)
    checked fold by fold against a host replay (SVS_POA_VERIFY_GRAPH=1: rank
    order, row tables, consensus, MSA), pruned retries included, also with a
    64-entry LDS part of the sort's DFS stack so that deep DFS paths spill to
    the task block; and with the host graphs (SVS_POA_HOST_GRAPH=1), their
    row tables completed on the device and checked table for table against
    the host's export (SVS_POA_VERIFY_PREP=1)."""
    import os
    from svscope_amd import synth
    from svscope_amd.poa import poa_batch
    cases = helpers.random_cases(31, 40, max_seqs=10, max_len=260, edits=20)
    cases += [synth.make_window(w, 12, 1500)[0] for w in range(2)]
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        got = poa_batch(cases)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    for seqs, g in zip(cases, got):
        assert g == oracle_poa(seqs, 1)


@pytest.mark.parametrize("env", [
    {"SVS_POA_WPJ": "2"},
    {"SVS_POA_WPJ": "4"},
    {"SVS_POA_WPJ": "8"},
    {"SVS_POA_STRIP_GLOBAL_POOL": "1", "SVS_POA_WPJ": "4"},
])
def test_short_graph_strip_handoff(env):
    """Many reads aligned to graphs of 1-7 rows (a first read of 1-7 bases):
    each strip's carries are one partial 8-row line, published at the strip's
    end, and the next strip's wave is already spinning on it.  The consumer
    reads carries with scalar loads, which are not ordered behind the
    producer's vector stores by the workgroup-scope release alone; a stale
    carry moved the single base of the first read to another column of the
    MSA (profiles/r04_i4/pytest_gpu.log, env19).  Several thousand such
    handoffs per kernel instance, every one against the oracle."""
    import os
    import random
    from svscope_amd.poa import poa_batch
    rnd = random.Random(44)
    cases = []
    for _ in range(1500):
        first = "".join(rnd.choice("ACGT") for _ in range(rnd.randint(1, 7)))
        second = "".join(rnd.choice("ACGT") for _ in range(rnd.randint(130, 640)))
        cases.append([first, second])
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        got = poa_batch(cases)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    bad = [i for i, (seqs, g) in enumerate(zip(cases, got)) if g != oracle_poa(seqs, 1)]
    assert not bad, (len(bad), cases[bad[0]])


@pytest.mark.parametrize("slack,retries", [("0.05", None), ("-0.3", True)])
def test_pruning_stats_and_exactness(slack, retries):
    """The strip kernel's exact pruning on config-3-like windows: the oracle's
    MSA and consensus, fewer cells evaluated than the full matrix, and with a
    bound above every optimum (negative slack) every pruned job retried."""
    import os
    from svscope_amd import synth
    from svscope_amd.poa import poa_batch
    wins = [synth.make_window(w, 10, 3000)[0] for w in range(3)]
    old = os.environ.get("SVS_POA_PRUNE_SLACK")
    os.environ["SVS_POA_PRUNE_SLACK"] = slack
    try:
        got, st = poa_batch(wins, return_stats=True)
    finally:
        if old is None:
            os.environ.pop("SVS_POA_PRUNE_SLACK", None)
        else:
            os.environ["SVS_POA_PRUNE_SLACK"] = old
    for seqs, g in zip(wins, got):
        assert g == oracle_poa(seqs, 1)
    if retries:
        assert st["prune_retries"] > 0
    else:
        assert st["cells_computed"] < 0.6 * st["dp_cells"], st
    assert st["prep_jobs"] > 0, st  # the device completed the row tables
    assert st["fold_jobs"] > 0, st  # and folded the alignments into its graphs
    # the graph arena's footprint is reported (DevArena accounting)
    assert 0 < st["dgraph_peak_bytes"] <= st["dgraph_reserved_bytes"], st
    # the DP busy time is the union of the launch intervals: no longer than
    # their sum, no shorter than the sum spread over the task groups' streams
    assert 0 < st["kernel_busy_ms"] <= st["kernel_ms"] * (1 + 1e-6), st
    assert st["kernel_busy_ms"] >= st["kernel_ms"] / 4 - 1e-3, st


def test_wide_slot_jobs_share_pruned_launches():
    """Jobs whose pool slots go past the pruning kernel's 31 liveness bits get
    no bound of their own (kPruneAll) yet run in the same pruning launches as
    bounded jobs; both give the oracle's result.  The test hook numbers the
    slots of graphs with >= 1500 rows from 40 up."""
    import os
    from svscope_amd import synth
    from svscope_amd.poa import poa_batch
    wide = [synth.make_window(w, 8, 2500)[0] for w in range(2)]
    # graphs under 1500 rows: bounded (pruned) jobs in the same launches
    small = [synth.make_window(w, 8, 900)[0] for w in range(10, 14)]
    small += helpers.random_cases(77, 20, max_seqs=10, max_len=260, edits=20)
    cases = [c for pair in zip(small[:2], wide) for c in pair] + small[2:]
    # (host graphs: the slot-numbering hook lives in their planner)
    env = {"SVS_POA_TEST_WIDE_SLOTS": "1500", "SVS_POA_VERIFY_PREP": "1", "SVS_POA_HOST_GRAPH": "1"}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        got, st = poa_batch(cases, return_stats=True)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    for seqs, g in zip(cases, got):
        assert g == oracle_poa(seqs, 1)
    assert st["cells_computed"] < st["dp_cells"], st  # the bounded jobs were pruned


def test_device_graphs_verified_against_host_replay():
    """Device-resident graphs (poa_fold.hip) on the random edge cases and on
    longer windows: every fold checked against a host PoaGraph replay (rank
    order, lite and completed row tables, consensus, MSA rows), and the
    results equal to the oracle's."""
    import os
    from svscope_amd import synth
    from svscope_amd.poa import poa_batch
    cases = helpers.random_cases(211, 300) + helpers.random_cases(9, 30, max_seqs=12, max_len=300, edits=25)
    cases += [synth.make_window(w, 24, 2000)[0] for w in range(2)]
    cases += [["", "ACGT", "", "ACGA", ""], ["", ""], ["A"], ["ACGTACGT"] * 5]
    os.environ["SVS_POA_VERIFY_GRAPH"] = "1"
    try:
        got = poa_batch(cases)
    finally:
        os.environ.pop("SVS_POA_VERIFY_GRAPH", None)
    for seqs, g in zip(cases, got):
        assert g == oracle_poa(seqs, 1), seqs



@pytest.mark.parametrize("mode", ["device", "host"])
def test_wide_traceback_codes_match_oracle(mode):
    """32-bit traceback codes (TbFmt<uint32_t>: graphs with a node of more than
    31 in-edges) on every launch (SVS_POA_FORCE_WIDE):
    the wide kernel variants, their in-degree from pstart and the 12-bit
    in-edge fields of the traceback, on the random edge cases and synthetic
    windows, device graphs (checked fold by fold against a host replay) and
    host graphs, give the oracle's consensus and MSA."""
    import os
    from svscope_amd import synth
    from svscope_amd.poa import poa_batch
    cases = helpers.random_cases(31, 120) + helpers.random_cases(32, 12, max_seqs=12, max_len=300, edits=25)
    cases += [synth.make_window(w, 16, 1500)[0] for w in range(2)]
    env = {"SVS_POA_FORCE_WIDE": "1"}
    env.update({"SVS_POA_VERIFY_GRAPH": "1"} if mode == "device" else {"SVS_POA_HOST_GRAPH": "1"})
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        got, st = poa_batch(cases, return_stats=True)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    for seqs, g in zip(cases, got):
        assert g == oracle_poa(seqs, 1), seqs
    assert st["wide_launches"] == st["launches"] > 0, st
