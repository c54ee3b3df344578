"""Host-side pieces of bench.py and localGraph_npz (no GPU): the --gpus N
launcher, and the crash/--Continue journal of localGraph_npz (records written
per completed batch, SVscope.py:220-236)."""
import argparse
import json
import os
import subprocess
import sys

import numpy as np

from svscope_amd import local_graph, synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_gpus_launches_one_rank_per_gpu(tmp_path):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    subprocess.check_call([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--probe-env",
                           str(tmp_path)], env=env, timeout=300)
    got = sorted(json.load(open(tmp_path / f"rank{r}.json")).items() for r in range(2))
    seen = [dict(x) for x in got]
    assert sorted(d["RANK"] for d in seen) == ["0", "1"]
    assert sorted(d["LOCAL_RANK"] for d in seen) == ["0", "1"]
    assert {d["WORLD_SIZE"] for d in seen} == {"2"}
    assert {d["MASTER_ADDR"] for d in seen} == {"127.0.0.1"}


def _oracle_batches(rows, batch_size=512, context=None, depth=4):
    from oracle import decision_oracle
    for k in range(0, len(rows), batch_size):
        yield [decision_oracle.tdscope_npz(r[4], r[0], np.asarray(r[1]), r[2], r[3]) for r in rows[k:k + batch_size]]


def _crashing_batches(limit):
    def gen(rows, batch_size=512, context=None, depth=4):
        for k, recs in enumerate(_oracle_batches(rows, batch_size)):
            if k == limit:
                raise RuntimeError("simulated crash")
            yield recs
    return gen


def _expected(rows):
    from oracle import decision_oracle
    return local_graph.sort_lines([decision_oracle.record_line(x) for x in
                                   (r for b in _oracle_batches(rows, 1000) for r in b)])


def test_local_graph_journal_survives_crash_and_continue_resumes(tmp_path, monkeypatch):
    rows = [synth.make_window(w, 6, 150) for w in range(9)]
    synth.save_npz(str(tmp_path / "T1.vs.N1.b0.npz"), rows)
    args = argparse.Namespace(TSampleID="T1", NSampleID="N1", savedir=str(tmp_path), Continue=False, batch=2)
    monkeypatch.setattr(local_graph, "iter_batches", _crashing_batches(2))
    try:
        local_graph.localGraph_npz(args)
    except RuntimeError:
        pass
    path = tmp_path / "T1.vs.N1.TandemRepeat.Raw.bed"
    partial = open(path).read().splitlines()
    assert len(partial) == 4  # two completed batches of two, flushed before the crash
    # --Continue runs only what is missing and sorts the whole file
    seen = []

    def counting(rows_, batch_size=512, context=None, depth=4):
        seen.extend(rows_)
        yield from _oracle_batches(rows_, batch_size)
    monkeypatch.setattr(local_graph, "iter_batches", counting)
    args.Continue = True
    local_graph.localGraph_npz(args)
    assert len(seen) == 5
    assert open(path).read().splitlines() == _expected(rows)


def test_local_graph_merges_stale_rank_journals(tmp_path, monkeypatch):
    """An interrupted N > 1 run leaves <out>.part<rank> journals; the next
    --Continue run folds them into the output (a torn last line is dropped)
    and runs only the windows none of them holds."""
    from oracle import decision_oracle
    rows = [synth.make_window(w, 6, 150) for w in range(6)]
    synth.save_npz(str(tmp_path / "T1.vs.N1.b0.npz"), rows)
    path = tmp_path / "T1.vs.N1.TandemRepeat.Raw.bed"
    recs = [decision_oracle.record_line(x) for b in _oracle_batches(rows, 1) for x in b]
    open(path, "w").write(recs[0] + "\n")
    open(str(path) + ".part0", "w").write(recs[1] + "\n" + recs[2] + "\n")
    open(str(path) + ".part1", "w").write(recs[3] + "\n" + recs[4][:20])
    seen = []

    def counting(rows_, batch_size=512, context=None, depth=4):
        seen.extend(rows_)
        yield from _oracle_batches(rows_, batch_size)
    monkeypatch.setattr(local_graph, "iter_batches", counting)
    args = argparse.Namespace(TSampleID="T1", NSampleID="N1", savedir=str(tmp_path), Continue=True, batch=4)
    local_graph.localGraph_npz(args)
    assert len(seen) == 2
    assert not any(x.startswith(path.name + ".part") for x in os.listdir(tmp_path))
    assert open(path).read().splitlines() == _expected(rows)


def test_rank_cpu_plan_splits_the_job_share():
    """Eight ranks on one node (WORLD_SIZE=8): each gets a disjoint contiguous
    slice of the job's CPUs and share // 8 (>= 2) engine pool threads, so the
    ranks together stay within the job's CPU share."""
    from svscope_amd import hostcpu
    cpus = list(range(256))
    slices = [hostcpu.rank_cpu_plan(r, 8, cpus=cpus, share=16) for r in range(8)]
    assert {t for _, t in slices} == {2}
    assert sorted(c for s, _ in slices for c in s) == cpus
    assert all(s == list(range(32 * r, 32 * r + 32)) for r, (s, _) in enumerate(slices))
    assert hostcpu.rank_cpu_plan(0, 1, cpus=cpus, share=16) == (cpus, 16)
    assert hostcpu.rank_cpu_plan(1, 2, cpus=cpus, share=128)[1] == 16  # capped at 16
    # apply() in a fresh process: the rank's env, pinned, SVS_HOST_THREADS exported
    code = ("import os; from svscope_amd import hostcpu; n = hostcpu.apply(); "
            "print(n, os.environ['SVS_HOST_THREADS'], len(os.sched_getaffinity(0)))")
    env = dict(os.environ, LOCAL_RANK="3", LOCAL_WORLD_SIZE="8", WORLD_SIZE="8", OMP_NUM_THREADS="16")
    env.pop("SVS_HOST_THREADS", None)
    out = subprocess.check_output([sys.executable, "-c", code], env=env, cwd=ROOT, timeout=120).decode().split()
    n_aff = len(os.sched_getaffinity(0))
    assert out[:2] == ["2", "2"] and int(out[2]) == max(1, n_aff // 8)


def test_dp_busy_union_matches_brute_force():
    """kernel_busy_ms (bench.py roofline.dp_busy) is the union of the DP
    launches' intervals, accumulated as launches complete in any order
    (svscope_amd/csrc/svs_busy.hpp through tests/cpp/busy_union_emu.cpp),
    checked against a sort-and-sweep union after every added interval:
    disjoint, nested, touching, duplicate and empty intervals, two streams'
    overlapping launches completing out of order."""
    import ctypes
    import random
    src = os.path.join(ROOT, "tests", "cpp", "busy_union_emu.cpp")
    hdr = os.path.join(ROOT, "svscope_amd", "csrc", "svs_busy.hpp")
    lib_path = os.path.join(ROOT, "tests", "build", "libbusy_union_emu.so")
    os.makedirs(os.path.dirname(lib_path), exist_ok=True)
    if not os.path.exists(lib_path) or os.path.getmtime(lib_path) < max(os.path.getmtime(src), os.path.getmtime(hdr)):
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-o", lib_path, src])
    lib = ctypes.CDLL(lib_path)
    D = ctypes.POINTER(ctypes.c_double)
    lib.emu_busy_union.argtypes = [D, D, ctypes.c_int, D]

    def brute(iv):
        tot, cur = 0.0, None
        for a, b in sorted(iv):
            if cur is None or a > cur[1]:
                if cur:
                    tot += cur[1] - cur[0]
                cur = [a, b]
            else:
                cur[1] = max(cur[1], b)
        return tot + (cur[1] - cur[0] if cur else 0.0)

    rng = random.Random(7)
    cases = [[(0, 1), (2, 3), (1, 2)], [(0, 10), (2, 3), (4, 5)], [(5, 6), (5, 6), (3, 3)], [(3, 4), (0, 1), (1, 3)]]
    for _ in range(300):
        n = rng.randint(1, 40)
        iv = []
        for _ in range(n):
            a = rng.choice([rng.uniform(0, 100), float(rng.randint(0, 20))])
            iv.append((a, a + rng.choice([0.0, rng.uniform(0, 15), float(rng.randint(0, 5))])))
        cases.append(iv)
    # two DP streams: each stream's launches back to back, the streams
    # overlapping, reported in completion order
    for _ in range(50):
        iv = []
        for s in range(2):
            t = rng.uniform(0, 5)
            for _ in range(20):
                d = rng.uniform(1, 4)
                iv.append((t, t + d))
                t += d + rng.uniform(0, 3)
        iv.sort(key=lambda x: x[1])
        cases.append(iv)
    for iv in cases:
        n = len(iv)
        lo = (ctypes.c_double * n)(*[a for a, _ in iv])
        hi = (ctypes.c_double * n)(*[b for _, b in iv])
        out = (ctypes.c_double * n)()
        lib.emu_busy_union(lo, hi, n, out)
        for k in range(n):
            assert abs(out[k] - brute(iv[:k + 1])) < 1e-9, (iv[:k + 1], out[k])


def test_block_arena_never_hands_out_overlapping_blocks():
    """The device graph arena's block logic (svscope_amd/csrc/
    svs_block_arena.hpp) under a fake chunk allocator, at limits
    between 1 and 100 GiB, most of them giving a chunk size that the old
    arena did not round to a power of two: random task-sized allocations and
    frees run it past its limit, so chunk tails are filed, split_larger
    halves blocks and try_alloc returns null; no live block may overlap
    another or leave its chunk (tests/cpp/block_arena_emu.cpp)."""
    import ctypes
    src = os.path.join(ROOT, "tests", "cpp", "block_arena_emu.cpp")
    hdr = os.path.join(ROOT, "svscope_amd", "csrc", "svs_block_arena.hpp")
    lib_path = os.path.join(ROOT, "tests", "build", "libblock_arena_emu.so")
    os.makedirs(os.path.dirname(lib_path), exist_ok=True)
    if not os.path.exists(lib_path) or os.path.getmtime(lib_path) < max(os.path.getmtime(src), os.path.getmtime(hdr)):
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-o", lib_path, src])
    lib = ctypes.CDLL(lib_path)
    lib.emu_block_arena.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int,
                                    ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
    GiB = 1 << 30
    total_null = 0
    for limit in (64 << 20, 300 << 20, 1 * GiB, int(5.3 * GiB), 6 * GiB, int(20.7 * GiB), 48 * GiB, int(63.9 * GiB), 100 * GiB):
        for seed in range(3):
            n_null, n_checked = ctypes.c_int(), ctypes.c_int()
            bad = lib.emu_block_arena(limit, seed, 20000, ctypes.byref(n_null), ctypes.byref(n_checked))
            assert bad == 0, (limit, seed, bad)
            assert n_checked.value > 1000
            total_null += n_null.value
    assert total_null > 0  # the limit was reached: split_larger and null returns ran


def test_bench_deals_one_global_window_set_by_lpt(monkeypatch):
    """bench.py --gpus N: the ranks share one global set
    of N*K*B windows dealt by local_graph.lpt_owner over N*L^2, each rank
    generating every N-th window, exchanging their costs through the
    rendezvous store and generating the owned windows it lacks.  Two ranks as
    threads over one in-process store (small windows): the deal covers every
    id once, equals shard_lpt over the whole set, and every owned row is that
    window."""
    import threading
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    import bench
    monkeypatch.setattr(bench, "N_READS", 6)
    monkeypatch.setattr(bench, "REF_LEN", 160)
    world, K, B = 2, 3, 5
    store = dist.HashStore()
    got = {}

    def run(r):
        got[r] = bench.deal_global(world, r, K, B, 1, dist.PrefixStore("svs_bench_deal", store))
    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert set(got) == {0, 1}
    allrows = [synth.make_window(w, 6, 160) for w in range(world * K * B)]
    owner = local_graph.shard_lpt(allrows, world)
    for r in range(world):
        ids, rows, per_n, per_cost = got[r]
        assert ids == [w for w in range(world * K * B) if owner[w] == r]
        assert [local_graph.window_key(x) for x in rows] == [synth.window_key(w, 160) for w in ids]
        assert all(list(x[0]) == list(allrows[w][0]) for w, x in zip(ids, rows))
        assert per_n == [owner.count(k) for k in range(world)]
    assert sorted(got[0][0] + got[1][0]) == list(range(world * K * B))


def test_bench_oracle_check_finds_windows_among_sorted_lines(tmp_path, monkeypatch):
    """record_digests locates the fixture's windows among rank 0's gathered,
    sorted lines by chrom / start / end, whatever rank produced them."""
    import hashlib
    sys.path.insert(0, ROOT)
    import bench
    gold = {"digests": [], "sparse_ids": [7], "sparse_digests": []}
    lines = []
    for w in range(10):
        line = synth.window_key(w, bench.REF_LEN) + "\t3\tX\tY|EMOutput"
        lines.append(line)
        if w < 4:
            gold["digests"].append(hashlib.sha256(line.encode()).hexdigest())
        if w == 7:
            gold["sparse_digests"].append(hashlib.sha256(line.encode()).hexdigest())
    gold["all"] = None
    path = tmp_path / "g.json"
    path.write_text(json.dumps(gold))
    monkeypatch.setattr(bench, "GOLDEN_DIGESTS", str(path))
    out = bench.record_digests(local_graph.sort_lines(lines[::-1]))
    assert out["match"] and out["windows"] == 4 and out["windows_checked"] == 5
    lines[2] = lines[2].replace("X", "Z")
    out = bench.record_digests(lines)
    assert not out["match"] and out["mismatched_windows"] == [2]
