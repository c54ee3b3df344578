"""The N > 1 path of localGraph_npz (svscope_amd/local_graph.py):
longest-first window sharding and the one all_gather of packed records,
rehearsed with world_size 2 on gloo (CPU).  The per-window decision is the
CPU oracle here (test infrastructure); on GPUs it is the HIP engine."""
import argparse
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from svscope_amd import local_graph, synth


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _oracle_run(rows, batch_size=512, context=None, stats=None):
    from oracle import decision_oracle
    return [decision_oracle.tdscope_npz(r[4], r[0], np.asarray(r[1]), r[2], r[3]) for r in rows]


def _oracle_batches(rows, batch_size=512, context=None, depth=4):
    for k in range(0, len(rows), batch_size):
        yield _oracle_run(rows[k:k + batch_size])


def _rank_main(rank, world, port, savedir, outdir):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    local_graph.iter_batches = _oracle_batches
    args = argparse.Namespace(TSampleID="T1", NSampleID="N1", savedir=savedir, Continue=False, batch=4)
    path = local_graph.localGraph_npz(args)
    import torch.distributed as dist
    dist.barrier()
    dist.destroy_process_group()
    if rank == 0:
        os.replace(path, os.path.join(outdir, "world.bed"))


def _write_bundles(d, rows):
    for k in range(0, len(rows), 5):
        arr = np.empty(len(rows[k:k + 5]), dtype=object)
        for i, r in enumerate(rows[k:k + 5]):
            arr[i] = r
        np.savez(os.path.join(d, f"part{k // 5}.npz"), DatSet=arr)


def test_shard_lpt_balanced_and_complete():
    rows = [synth.make_window(w, 4 + w % 5, 100 + 37 * (w % 7)) for w in range(40)]
    for world in (1, 2, 3, 8):
        owner = local_graph.shard_lpt(rows, world)
        assert len(owner) == len(rows) and set(owner) <= set(range(world))
        load = [0.0] * world
        for r, o in zip(rows, owner):
            load[o] += local_graph.window_cost(r)
        biggest = max(local_graph.window_cost(r) for r in rows)
        assert max(load) - min(load) <= biggest + 1e-9
        assert owner == local_graph.shard_lpt(rows, world)


def test_local_graph_world2_gloo_matches_single_process(tmp_path):
    rows = [synth.make_window(w, 6, 160) for w in range(12)]
    savedir = tmp_path / "bundles"
    savedir.mkdir()
    _write_bundles(str(savedir), rows)
    exp = local_graph.sort_lines([local_graph.record_line(x) for x in _oracle_run(rows)])
    port = _free_port()
    mp.start_processes(_rank_main, args=(2, port, str(savedir), str(tmp_path)), nprocs=2, join=True,
                       start_method="fork")
    got = [x.rstrip("\n") for x in open(tmp_path / "world.bed")]
    assert got == exp
