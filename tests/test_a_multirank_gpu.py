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
