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
