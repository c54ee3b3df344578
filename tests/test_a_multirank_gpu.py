"""The HIP engine under torch.distributed: localGraph_npz
with two ranks on the one GPU of the box (SVS_DEVICE=0, record gather over
gloo), each rank a fresh process started by torch.distributed.run before
anything touches the GPU (this module sorts first, so the pytest process has
not initialised the GPU when it starts them).  The real DecisionSession runs
each rank's LPT shard of 24 config-3 windows (64 reads x 3 kb, bench window
ids 0..23); rank 0's gathered, sorted Raw.bed must hold exactly the oracle's
records (tests/golden/bench_config3_digests.json) in sort -k1,1 -k2,2n
order, and the shards must split the windows between the ranks."""
import hashlib
import json
import os
import socket
import subprocess
import sys

import pytest

from svscope_amd import local_graph, synth

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_local_graph_npz_two_ranks_on_gpu(tmp_path):
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "bench_config3_digests.json")))
    n = 24
    rows = [synth.make_window(w, 64, 3000) for w in range(n)]
    savedir = tmp_path / "bundles"
    savedir.mkdir()
    for k in range(0, n, 8):
        synth.save_npz(str(savedir / f"part{k // 8}.npz"), rows[k:k + 8])
    env = dict(os.environ, SVS_DEVICE="0", SVS_DIST_BACKEND="gloo", PYTHONPATH=ROOT)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "multirank_main.py"), str(savedir), str(tmp_path)]
    p = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    lines = [x.rstrip("\n") for x in open(savedir / "T1.vs.N1.TandemRepeat.Raw.bed")]
    assert lines == local_graph.sort_lines(lines)
    got = sorted(hashlib.sha256(x.encode()).hexdigest() for x in lines)
    assert got == sorted(gold["digests"][:n])
    shards = [open(tmp_path / f"rank{r}.txt").read().split("\n") for r in range(2)]
    assert all(shards) and sorted(shards[0] + shards[1]) == sorted(local_graph.window_key(r) for r in rows)
    # the per-rank journals are gone once rank 0 has the records
    assert not [x for x in os.listdir(savedir) if ".part" in x]


def test_bench_two_ranks_on_gpu_runs_the_multi_gpu_path(tmp_path):
    """bench.py --gpus 2 rehearsed on the box's one GPU (SVS_DIST_BACKEND=gloo,
    SVS_DEVICE=0): one global set of 2 x 2 x 8 config-3
    windows dealt by LPT, each rank's shard through its own session, the
    record lines gathered to rank 0 and sorted inside the timed region.  The
    JSON line must report both ranks (windows, LPT cost, elapsed, the gather)
    and rank 0's gathered records must match the oracle's digests of windows
    0..31."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(SVS_DEVICE="0", SVS_DIST_BACKEND="gloo", PYTHONPATH=ROOT)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--batch", "8",
           "--warmup", "1", "--depth", "2", "--cpu-sample", "0", "--gen-procs", "4"]
    p = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=400)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    line = [x for x in p.stdout.splitlines() if x.startswith("{")][-1]
    print(line)
    out = json.loads(line)
    assert out["n_gpus"] == 2 and out["value"] > 0
    r = out["ranks"]
    assert sum(r["windows"]) == 32 and r["windows"] == r["lpt_windows"] and min(r["windows"]) > 0
    assert len(r["elapsed_s"]) == 2 and r["gather_and_sort_s"] >= 0 and len(r["lpt_cost"]) == 2
    assert out["oracle_check"]["match"] and out["oracle_check"]["windows"] == 32
    assert 0 < out["roofline"]["frac"] < 1
