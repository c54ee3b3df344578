"""GPU parity of the whole per-window path (Decision / TDscope_npz): records
identical to the reference's own records (goldens) and to the CPU oracle."""
import hashlib
import json
import os

import numpy as np
import pytest

from oracle import decision_oracle

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden", "decision_goldens.json")


@pytest.mark.parametrize("env", [{}, {"SVS_POA_VERIFY_GRAPH": "1"}, {"SVS_DEVICE_FEATURES": "0"}])
def test_decision_batch_matches_reference_goldens(env, monkeypatch):
    """The reference's own records (full-deletion read, gate failures,
    germline-only window, empty flanks): with the window's feature selection
    on the device (default), with it checked against the host's selection from
    the returned MSA rows (SVS_POA_VERIFY_GRAPH=1), and on the host
    (SVS_DEVICE_FEATURES=0)."""
    from svscope_amd.decision_maker import DecisionBatch
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    cases = json.load(open(GOLD))
    wins = [(c["TDRecord"], c["sequenceList"], np.array(c["ReadIDs"]), c["flank_5"], c["flank_3"]) for c in cases]
    for c, rec in zip(cases, DecisionBatch(wins)):
        assert "\t".join(str(x) for x in rec) == c["line"], c["kind"]


def test_single_window_decision_signature():
    from svscope_amd.decision_maker import Decision
    c = json.load(open(GOLD))[0]
    rec = Decision(c["TDRecord"], c["sequenceList"], np.array(c["ReadIDs"]), c["flank_5"], c["flank_3"])
    assert "\t".join(str(x) for x in rec) == c["line"]


def test_feature_selection_on_gpu_matches_reference():
    from svscope_amd.data_scanner import MSAFeatureSelection
    for c in json.load(open(GOLD)):
        if not c["features"]:
            continue
        enc, feat, rid = MSAFeatureSelection(c["sequenceList"], c["flank_5"], c["flank_3"], np.array(c["ReadIDs"]))
        assert list(enc.shape) == c["features"]["encoded_shape"]
        assert feat.tolist() == c["features"]["seqdatamx"]
        assert list(map(str, rid)) == c["features"]["read_ids"]


def test_config1_and_config2_windows_match_oracle():
    """configs[0]: one 16-read x 2 kb window; configs[1]-shaped: 32 reads x 2 kb."""
    from svscope_amd import synth
    from svscope_amd.som_td_detector import TDscope_npz_batch
    rows = synth.make_windows(config=1) + [synth.make_window(3, 32, 2000)]
    for r, g in zip(rows, TDscope_npz_batch(rows)):
        exp = decision_oracle.tdscope_npz(r[4], r[0], np.asarray(r[1]), r[2], r[3])
        assert decision_oracle.record_line(g) == decision_oracle.record_line(exp)


def test_local_graph_npz_end_to_end(tmp_path):
    from svscope_amd import synth
    from svscope_amd.local_graph import main
    rows = [synth.make_window(w, 10, 400) for w in range(6)]
    synth.save_npz(str(tmp_path / "T1.vs.N1.TandemRepeat.batch0.npz"), rows[:4])
    synth.save_npz(str(tmp_path / "T1.vs.N1.TandemRepeat.batch1.npz"), rows[4:])
    main(["-t", "T1", "-n", "N1", "-s", str(tmp_path), "--batch", "4"])
    lines = open(tmp_path / "T1.vs.N1.TandemRepeat.Raw.bed").read().splitlines()
    exp = sorted((decision_oracle.record_line(decision_oracle.tdscope_npz(r[4], r[0], np.asarray(r[1]), r[2], r[3]))
                  for r in rows), key=lambda l: (l.split("\t")[0], int(l.split("\t")[1]), l))
    assert lines == exp
    # --Continue skips everything already written
    main(["-t", "T1", "-n", "N1", "-s", str(tmp_path), "-C"])
    assert open(tmp_path / "T1.vs.N1.TandemRepeat.Raw.bed").read().splitlines() == exp


def _oracle_record(r):
    return decision_oracle.record_line(decision_oracle.tdscope_npz(r[4], r[0], np.asarray(r[1]), r[2], r[3]))


def test_config3_windows_match_oracle():
    """configs[2] at full size: two 64-read x 3 kb windows (one somatic
    insertion, one deletion) through the whole GPU pipeline (MSA POA with exact
    pruning, features, EM, consensus POA) against the CPU oracle, record for
    record (the oracle runs in two processes, about 25 s each)."""
    import multiprocessing as mp
    from svscope_amd import synth
    from svscope_amd.som_td_detector import TDscope_npz_batch
    rows = [synth.make_window(w, 64, 3000) for w in (0, 1)]
    got = [decision_oracle.record_line(g) for g in TDscope_npz_batch(rows)]
    with mp.get_context("fork").Pool(2) as pool:
        exp = pool.map(_oracle_record, rows)
    assert got == exp


def test_config3_batch_invariants():
    """Size-independent properties at full config-3 size (64 reads x 3 kb):
    the continuous-batching engine gives the same records whatever the batch
    composition and order (32 windows at once, again, then reversed in two
    halves), and every EMOutput record's read ids are window read ids, each
    in at most one cluster."""
    from svscope_amd import synth
    from svscope_amd.som_td_detector import TDscope_npz_batch
    rows = [synth.make_window(w, 64, 3000) for w in range(100, 132)]
    first = [decision_oracle.record_line(g) for g in TDscope_npz_batch(rows)]
    again = [decision_oracle.record_line(g) for g in TDscope_npz_batch(rows)]
    assert first == again
    rev = rows[::-1]
    split = TDscope_npz_batch(rev[:11]) + TDscope_npz_batch(rev[11:])
    assert [decision_oracle.record_line(g) for g in split][::-1] == first
    n_em = 0
    for r, line in zip(rows, first):
        f = line.split("\t")
        if not f[-1].endswith("|EMOutput"):
            continue
        n_em += 1
        ids = set(map(str, r[1]))
        seen = []
        for field in (f[4], f[7]):
            for cluster in field.split(";"):
                seen += [x for x in cluster.split(",") if x]
        assert set(seen) <= ids and len(seen) == len(set(seen)), line[:200]
    assert n_em > 0


def test_decision_session_streams_batches_out_of_order():
    """The streaming session (svs_decision_session_*): golden windows split
    over several batches, one with no gated window, submitted back to back and
    waited for out of order, give the reference's records; a closed session
    refuses work and an unknown ticket fails loudly."""
    from svscope_amd import _abi
    from svscope_amd.decision_maker import DecisionSession
    cases = json.load(open(GOLD))
    wins = [(c["TDRecord"], c["sequenceList"], np.array(c["ReadIDs"]), c["flank_5"], c["flank_3"]) for c in cases]
    lines = [c["line"] for c in cases]
    gate = [k for k, c in enumerate(cases) if c["kind"] in ("one_tag", "few_reads")]
    assert gate
    # batch 2 holds only windows that fail the gate (never reach the engine)
    order = [list(range(0, 5)), gate, [k for k in range(5, len(cases)) if k not in gate]]
    s = DecisionSession()
    tickets = [s.submit([wins[k] for k in part]) for part in order]
    got = {}
    for t in reversed(tickets):
        got[t] = s.wait(t)
    st = s.stats()
    assert st["msa_tasks"] > 0 and st["poa"]["launches"] > 0
    for t, part in zip(tickets, order):
        assert ["\t".join(str(x) for x in r) for r in got[t]] == [lines[k] for k in part]
    with pytest.raises(_abi.SvsError):
        _abi.check(s.lib.svs_decision_session_wait(s.handle, 10 ** 6, ctypes_ptr()), "wait")
    s.close()
    s.close()  # idempotent


def ctypes_ptr():
    import ctypes
    return ctypes.byref(ctypes.c_void_p())


def test_decision_session_config3_matches_batch_path():
    """Full-size config-3 windows through the session with batches in flight
    (the bench's path) equal the one-call batch path record for record."""
    from collections import deque
    from svscope_amd import synth
    from svscope_amd.decision_maker import DecisionSession
    from svscope_amd.local_graph import _window
    from svscope_amd.som_td_detector import TDscope_npz_batch
    rows = [synth.make_window(w, 64, 3000) for w in range(200, 224)]
    exp = [decision_oracle.record_line(g) for g in TDscope_npz_batch(rows)]
    got = []
    with DecisionSession() as s:
        q = deque()
        for k in range(0, len(rows), 5):
            q.append(s.submit([_window(r) for r in rows[k:k + 5]]))
            if len(q) >= 3:
                got += s.wait(q.popleft())
        while q:
            got += s.wait(q.popleft())
    assert [decision_oracle.record_line(g) for g in got] == exp


def test_decision_session_bad_batch_is_isolated():
    """A batch whose seq_byte_start is not monotone fails its own submit on the
    caller's thread (SVS_E_INVALID); the good batches before and after it still
    return the reference's records, and waiting twice for a ticket fails
    instead of hanging."""
    import ctypes
    from svscope_amd import _abi
    from svscope_amd.decision_maker import DecisionSession, _gate, _pack_windows
    cases = json.load(open(GOLD))
    wins = [(c["TDRecord"], c["sequenceList"], np.array(c["ReadIDs"]), c["flank_5"], c["flank_3"]) for c in cases]
    lines = [c["line"] for c in cases]
    s = DecisionSession()
    t1 = s.submit(wins[:4])
    # the same windows, packed, with two sequence starts swapped
    _, gated = _gate(wins[4:8])
    wpk, starts, blob, txt, tag_arr = _pack_windows(wins[4:8], gated, "tumor")
    bad = starts.copy()
    bad[2], bad[3] = starts[3], starts[2]
    ticket = ctypes.c_int64()
    with pytest.raises(_abi.SvsError, match="monotone"):
        _abi.check(s.lib.svs_decision_session_submit(
            s.handle, len(gated), wpk, bad.ctypes.data_as(ctypes.c_void_p), blob, txt,
            tag_arr.ctypes.data_as(ctypes.c_void_p), ctypes.byref(ticket)), "svs_decision_session_submit")
    t2 = s.submit(wins[4:9])
    assert ["\t".join(str(x) for x in r) for r in s.wait(t1)] == lines[:4]
    assert ["\t".join(str(x) for x in r) for r in s.wait(t2)] == lines[4:9]
    with pytest.raises(_abi.SvsError, match="already waited"):
        _abi.check(s.lib.svs_decision_session_wait(s.handle, ctypes.c_int64(t2), ctypes_ptr()), "wait")
    s.close()


def test_bench_windows_match_oracle_digests():
    """bench.py's own workload pinned against the CPU oracle: its first 256
    timed windows (config 3: 64 reads x 3 kb, window ids 0..255) through the
    streaming session exactly as bench.py runs them (batches of 64, 4 in
    flight), record for record against the SHA-256 of the oracle's Raw.bed
    line (tests/golden/bench_config3_digests.json, gen_bench_goldens.py)."""
    import hashlib
    from collections import deque
    from svscope_amd import synth
    from svscope_amd.decision_maker import DecisionSession
    from svscope_amd.local_graph import _window, record_line
    gold = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "bench_config3_digests.json")))
    rows = [synth.make_window(w, 64, 3000) for w in range(gold["n"])]
    got = []
    with DecisionSession() as s:
        q = deque()
        for k in range(0, len(rows), 64):
            q.append(s.submit([_window(r) for r in rows[k:k + 64]]))
            if len(q) >= 4:
                got += s.wait(q.popleft())
        while q:
            got += s.wait(q.popleft())
    digests = [hashlib.sha256(record_line(r).encode()).hexdigest() for r in got]
    bad = [k for k, (a, b) in enumerate(zip(digests, gold["digests"])) if a != b]
    assert not bad, f"{len(bad)} windows differ from the oracle, first {bad[:8]}"
    assert hashlib.sha256("\n".join(digests).encode()).hexdigest() == gold["all"]


def _session_digests(rows, batch, depth=4):
    """Records of rows through one streaming DecisionSession (batches of
    `batch`, `depth` in flight, as bench.py and localGraph_npz run), as the
    SHA-256 of each Raw.bed line; and the session's statistics."""
    import hashlib
    from collections import deque
    from svscope_amd.decision_maker import DecisionSession
    from svscope_amd.local_graph import _window, record_line
    got = []
    with DecisionSession() as s:
        q = deque()
        for k in range(0, len(rows), batch):
            q.append(s.submit([_window(r) for r in rows[k:k + batch]]))
            if len(q) >= depth:
                got += s.wait(q.popleft())
        while q:
            got += s.wait(q.popleft())
        st = s.stats()
    return [hashlib.sha256(record_line(r).encode()).hexdigest() for r in got], st


def test_device_features_verified_on_config3_windows(monkeypatch):
    """Config-3 windows (64 reads x 3 kb, bench window ids 0..11) with the
    graphs replayed on the host fold by fold and the device's seqdatamx,
    read ids and cluster reads compared with the host's selection from the
    MSA rows (SVS_POA_VERIFY_GRAPH=1), and the records equal to the oracle's
    digests (tests/golden/bench_config3_digests.json)."""
    from svscope_amd import synth
    monkeypatch.setenv("SVS_POA_VERIFY_GRAPH", "1")
    gold = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "bench_config3_digests.json")))
    rows = [synth.make_window(w, 64, 3000) for w in range(12)]
    digests, st = _session_digests(rows, 6)
    assert digests == gold["digests"][:12]


@pytest.mark.parametrize("name,batch", [("config2", 16), ("harsh", 8)])
def test_unbenched_paths_match_oracle_digests(name, batch):
    """the paths bench.py does not run, pinned against the
    CPU oracle (tests/golden/gen_path_goldens.py): 64 config-2 windows (32
    reads x 2 kb) through the streaming session, and 24 windows of
    tools/prune_probe.py's harsh profile (15 % error, 1.5-2.5 kb insertions),
    where the exact pruning's bound misses and retried alignments must still
    give the oracle's records (the test asserts that retries ran)."""
    from svscope_amd import synth
    gold = json.load(open(os.path.join(os.path.dirname(__file__), "golden", f"{name}_digests.json")))
    kw = {k: tuple(v) if isinstance(v, list) else v for k, v in gold["make_window_kw"].items()}
    rows = [synth.make_window(w, gold["reads"], gold["ref_len"], **kw) for w in range(gold["n"])]
    digests, st = _session_digests(rows, batch)
    bad = [k for k, (a, b) in enumerate(zip(digests, gold["digests"])) if a != b]
    assert not bad, f"{len(bad)} windows differ from the oracle, first {bad[:8]}"
    assert len(digests) == gold["n"]
    if name == "harsh":
        assert st["poa"]["prune_retries"] > 0, st["poa"]


def test_session_reproduces_reference_records_at_baseline_sizes():
    """the HIP session's records equal the reference's own
    DecisionMaker.Decision records (tests/golden/reference_path_goldens.json,
    gen_reference_path_goldens.py: the reference's code run in the build
    container with the oracle POA standing in for pyspoa) for 16 config-3
    windows (64 reads x 3 kb), 16 config-2 windows (32 x 2 kb) and 4 windows of
    the harsh pruning profile, all in one streaming session.

    What this pins and what it does not: the reference's own Decision,
    MSAFeatureSelection, EMCluster and record code.  The POA inside those
    records is this repo's spoa restatement (oracle/spoa_oracle.cpp), not
    pyspoa (absent here), so POA and consensus parity with spoa itself stays
    unpinned by these goldens."""
    from svscope_amd import synth
    ref = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_path_goldens.json")))
    rows, want = [], []
    for w in ref["windows"]:
        s = ref["sets"][w["set"]]
        kw = {k: tuple(v) if isinstance(v, list) else v for k, v in s["make_window_kw"].items()}
        rows.append(synth.make_window(w["window"], s["reads"], s["ref_len"], **kw))
        want.append(w["digest"])
    assert len(rows) == 36
    digests, _ = _session_digests(rows, 12)
    bad = [(ref["windows"][k]["set"], ref["windows"][k]["window"]) for k, (a, b) in enumerate(zip(digests, want))
           if a != b]
    assert not bad, f"windows differ from the reference's records: {bad}"


def test_big_windows_mixed_into_config3_batch_match_oracle():
    """windows past the 64-read configs, a 600-read one
    (300 tumor + 300 normal, 1.2 kb) and a 320-read one (2 kb), mixed into a
    batch of config-3 windows (64 reads x 3 kb), through the whole GPU
    pipeline (MSA POA, features, EM beyond 256 reads, consensus POA): every
    record equals the CPU oracle's (big_window_digests.json,
    gen_big_window_goldens.py; the config-3 windows against
    bench_config3_digests.json)."""
    import hashlib
    from svscope_amd import synth
    from svscope_amd.decision_maker import DecisionSession
    from svscope_amd.local_graph import _window, record_line
    gdir = os.path.join(os.path.dirname(__file__), "golden")
    bench = json.load(open(os.path.join(gdir, "bench_config3_digests.json")))
    big = json.load(open(os.path.join(gdir, "big_window_digests.json")))["windows"]
    rows, want = [], []
    for w in range(6):
        rows.append(synth.make_window(w, 64, 3000))
        want.append(bench["digests"][w])
        if w in (1, 3):
            b = big[0] if w == 1 else big[1]
            rows.append(synth.make_window(b["window"], b["reads"], b["ref_len"]))
            want.append(b["sha256"])
    with DecisionSession() as s:
        got = s.wait(s.submit([_window(r) for r in rows]))
    digests = [hashlib.sha256(record_line(r).encode()).hexdigest() for r in got]
    bad = [k for k, (a, b) in enumerate(zip(digests, want)) if a != b]
    assert not bad, f"windows {bad} differ from the oracle"


@pytest.mark.parametrize("env,why", [({"SVS_POA_TEST_MAX_ROWS": "4000"}, "planner"),
                                     ({"SVS_POA_TEST_SORT_LDS_WORDS": "1800"}, "sort kernel"),
                                     ({"SVS_POA_TEST_MAX_BLOCK_BYTES": "2000000"}, "graph arena is full")])
def test_window_past_an_engine_limit_fails_alone(env, why):
    """a window that goes past an engine limit fails alone
    (status SVS_DEC_FAILED, decision_maker.WindowFailed naming it) while the
    other windows of its batch and of the session get the oracle's records.
    The device planner's row limit (SVS_POA_TEST_MAX_ROWS), or the LDS the
    sort kernel's node flags may take (SVS_POA_TEST_SORT_LDS_WORDS, ADVICE
    r03: a graph past it used to fail the whole launch), or the largest graph
    block the device arena hands out (SVS_POA_TEST_MAX_BLOCK_BYTES: the path a
    block past the arena's byte limit takes, ADVICE r04: it used to abort the
    session), is lowered for the test so that one 64-read x 3 kb window
    crosses it."""
    from svscope_amd import synth
    from svscope_amd.decision_maker import DecisionSession, WindowFailed
    from svscope_amd.local_graph import _window, record_line
    small = [synth.make_window(w, 8, 600) for w in range(40, 46)]
    big = synth.make_window(50, 64, 3000)
    rows = small[:3] + [big] + small[3:]
    os.environ.update(env)
    try:
        with DecisionSession() as s:
            t1 = s.submit([_window(r) for r in rows])
            t2 = s.submit([_window(r) for r in small])
            with pytest.raises(WindowFailed) as ei:
                s.wait(t1)
            again = s.wait(t2)
    finally:
        for k in env:
            os.environ.pop(k, None)
    e = ei.value
    assert list(e.failed) == [3] and why in e.failed[3], e.failed
    assert e.records[3] is None
    exp = [_oracle_record(r) for r in small]
    got = [record_line(x) for k, x in enumerate(e.records) if k != 3]
    assert got == exp
    assert [record_line(x) for x in again] == exp


def test_tasks_wait_for_a_full_graph_arena():
    """a task whose graph block does not fit only because other
    tasks hold the arena right now waits for a later launch instead of
    failing, so whether a window fails does not depend on timing.  With the
    context's graph arena held to 8 MiB (SVS_POA_TEST_ARENA_BYTES; one chunk,
    about three 32-read x 800-bp window tasks), 16 such windows cannot all
    hold their blocks at once: tasks are deferred (poa deferred_tasks > 0),
    none fails, and every record is the oracle's."""
    from svscope_amd import _abi, synth
    from svscope_amd.decision_maker import DecisionSession
    from svscope_amd.local_graph import _window, record_line
    rows = [synth.make_window(w, 32, 800) for w in range(300, 316)]
    os.environ["SVS_POA_TEST_ARENA_BYTES"] = str(8 << 20)
    try:
        ctx = _abi.Context(0)
        with DecisionSession(ctx) as s:
            t = s.submit([_window(r) for r in rows])
            recs = s.wait(t)
            st = s.stats()
    finally:
        os.environ.pop("SVS_POA_TEST_ARENA_BYTES", None)
    assert st["poa"]["deferred_tasks"] > 0, st["poa"]
    assert st["poa"]["dgraph_reserved_bytes"] <= 8 << 20
    assert [record_line(x) for x in recs] == [_oracle_record(r) for r in rows]


def test_consensus_prior_off_gives_the_same_records():
    """SVS_POA_CONS_PRIOR < 0 turns off the pruning prior of a window's
    consensus tasks (their first alignment then runs unpruned): the records
    of 16 config-3 windows (bench ids 0..15) are still the oracle's
    (tests/golden/bench_config3_digests.json), since the pruning is exact
    either way."""
    from svscope_amd import synth
    from svscope_amd.decision_maker import DecisionSession
    from svscope_amd.local_graph import _window, record_line
    gold = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "bench_config3_digests.json")))
    rows = [synth.make_window(w, 64, 3000) for w in range(16)]
    os.environ["SVS_POA_CONS_PRIOR"] = "-1"
    try:
        with DecisionSession() as s:
            recs = s.wait(s.submit([_window(r) for r in rows]))
    finally:
        os.environ.pop("SVS_POA_CONS_PRIOR", None)
    assert [hashlib.sha256(record_line(x).encode()).hexdigest() for x in recs] == gold["digests"][:16]
