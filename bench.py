#!/usr/bin/env python3
"""Benchmark of the SVScope localGraph hot path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]

One step = one pass of the hot path (window MSA POA -> feature selection ->
EM over K=1..9 -> per-cluster consensus POA -> 10-field record) over a batch of
B synthetic config-3 windows (64 reads x 3 kb, BASELINE.json configs[2],
generator of SURVEY.md §8(d)) per GPU.  For N > 1 the script runs as one
process per GPU under torch.distributed.run; every rank processes its own
windows (weak scaling), time = max over ranks.  Rank 0 prints one JSON line.

roofline: the dominant kernel is the POA DP (poa_strip_kernel); achieved =
algorithmic bytes (20 B per DP cell: the int32 H,E,F,O,Q planes of convex NW,
SURVEY.md §8(d)) x cells per launch / mean launch time, from HIP events on the
engine's POA stream.  traffic = measured HBM bytes per DP cell from the
committed rocprofv3 PMC summary (profiles/pmc_poa_traffic.json) x cells per
launch, else null.
cpu_baseline: the CPU oracle (C++ spoa restatement + numpy EM + literal
Decision) on a bounded sample of the same windows, one process per core.
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "candidate-windows/sec (64 reads × 3 kb) localGraph, 1/2/4/8 MI355X; % HBM roofline"
HBM_PEAK_GBS = 8000.0
BYTES_PER_CELL = 20
N_READS, REF_LEN = 64, 3000


def _gen(ws):
    from svscope_amd import synth
    return [synth.make_window(w, N_READS, REF_LEN) for w in ws]


def generate(ids, procs):
    chunks = [ids[i::procs] for i in range(procs)]
    with mp.get_context("fork").Pool(procs) as pool:
        parts = pool.map(_gen, chunks)
    by_id = {}
    for chunk, part in zip(chunks, parts):
        for w, row in zip(chunk, part):
            by_id[w] = row
    return [by_id[w] for w in ids]


def _oracle_window(row):
    from oracle import decision_oracle
    return decision_oracle.tdscope_npz(row[4], row[0], row[1], row[2], row[3])


def cpu_baseline(rows, cores):
    from oracle import spoa_oracle
    spoa_oracle._load()  # build/load before timing
    t = time.time()
    with mp.get_context("fork").Pool(cores) as pool:
        pool.map(_oracle_window, rows, chunksize=1)
    wall = time.time() - t
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": len(rows) / wall, "unit": "windows/s", "cores": cores, "kind": "port",
            "sample": f"{len(rows)} config-3 windows (64 reads x 3 kb), one per process; CPU oracle "
                      f"(C++ spoa-NW-convex restatement standing in for pyspoa, numpy EM, literal Decision); "
                      f"wall {wall:.1f}s",
            "cpu_model": model, "nproc": os.cpu_count()}


def pmc_traffic_per_cell():
    """Measured HBM bytes per DP cell of the POA kernel from the committed
    rocprofv3 PMC summary (FETCH_SIZE and WRITE_SIZE passes), or None."""
    path = os.path.join(ROOT, "profiles", "pmc_poa_traffic.json")
    if not os.path.exists(path):
        return None
    try:
        return float(json.load(open(path))["hbm_bytes_per_cell"])
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=int(os.environ.get("SVS_BENCH_BATCH", "4096")))
    ap.add_argument("--cpu-sample", type=int, default=-1, help="windows for the CPU baseline (-1 auto, 0 off)")
    ap.add_argument("--gen-procs", type=int, default=min(16, os.cpu_count() or 1))
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    # synthetic windows first: the generator pool forks before this process
    # touches the GPU
    B, K, W = args.batch, args.steps, args.warmup
    per_rank = (W + K) * B
    ids = list(range(rank * per_rank, (rank + 1) * per_rank))
    rows = generate(ids, max(1, args.gen_procs))
    batches = [rows[s * B:(s + 1) * B] for s in range(W + K)]

    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        os.environ["SVS_DEVICE"] = str(local)
        dist.init_process_group("nccl")

    from svscope_amd import _abi
    from svscope_amd.som_td_detector import TDscope_npz_batch
    ctx = _abi.default_context()

    for s in range(W):
        TDscope_npz_batch(batches[s], context=ctx)

    stats = []
    if dist is not None:
        import torch
        dist.barrier()
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    n_em = 0
    for s in range(W, W + K):
        recs = TDscope_npz_batch(batches[s], context=ctx, stats=stats)
        n_em += sum(1 for r in recs if str(r[-1]).endswith("|EMOutput"))
    if dist is not None:
        dist.barrier()
        torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    poa_stats = [st for name, st in stats if name in ("msa_poa", "consensus_poa", "decision_poa")]
    cells = sum(st["dp_cells"] for st in poa_stats)
    # cells the kernel evaluated (its exact pruning skips strip rows that cannot
    # reach the alignment's bound): the roofline is priced on these
    cells_done = sum(st.get("cells_computed", st["dp_cells"]) for st in poa_stats)
    retries = sum(st.get("prune_retries", 0) for st in poa_stats)
    kms = sum(st["kernel_ms"] for st in poa_stats)
    launches = sum(st["launches"] for st in poa_stats)
    host_ms = sum(st["host_graph_ms"] for st in poa_stats)
    wait_ms = sum(st.get("gpu_wait_ms", 0.0) for st in poa_stats)
    phases = {}
    for name, st in stats:
        if name == "phases":
            for k, v in st.items():
                phases[k] = round(phases.get(k, 0.0) + v, 3)
    achieved = cells_done * BYTES_PER_CELL / (kms * 1e-3) / 1e9 if kms > 0 else 0.0
    total_windows = B * K * world

    if rank == 0:
        cpu = None
        n_cpu = args.cpu_sample
        if n_cpu != 0 and world == 1:  # the CPU baseline is an N=1 figure
            cores = min(16, os.cpu_count() or 1)
            if n_cpu < 0:
                n_cpu = cores
            cpu = cpu_baseline(batches[W][:n_cpu], min(cores, n_cpu))
        value = total_windows / elapsed
        per_cell = pmc_traffic_per_cell()
        traffic = round(per_cell * cells_done / max(1, launches)) if per_cell is not None else None
        out = {
            "metric": METRIC,
            "value": round(value, 4),
            "unit": "windows/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": round(elapsed * 1e3 / K, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic (SURVEY.md §8(d) generator: ONT-like 8% error, somatic INS/DEL, seeded)",
            "config": {"workload": "config3: 64 reads x 3 kb candidate windows, localGraph end-to-end "
                                   "(MSA POA + features + EM K=1..9 + consensus POA)",
                       "windows_per_step_per_gpu": B, "reads_per_window": N_READS, "ref_len": REF_LEN,
                       "parallelism": f"window shards x{world}"},
            "roofline": {"bound": "hbm", "kernel": "poa_strip_kernel",
                         "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5),
                         "traffic": traffic,
                         "algorithmic_bytes_per_launch": int(cells_done * BYTES_PER_CELL / max(1, launches)),
                         "mean_launch_ms": round(kms / max(1, launches), 4)},
            "cpu_baseline": cpu,
            "breakdown": {"poa_cells": cells, "poa_cells_computed": cells_done, "prune_retries": retries,
                          "poa_kernel_ms": round(kms, 2), "poa_launches": launches,
                          "gcups": round(cells_done / (kms * 1e-3) / 1e9, 3) if kms else None,
                          "gcups_full_matrix_equivalent": round(cells / (kms * 1e-3) / 1e9, 3) if kms else None,
                          "host_graph_ms": round(host_ms, 1), "host_wait_for_gpu_ms": round(wait_ms, 1),
                          "em_output_windows": n_em,
                          "phases_s": phases,
                          "em_dtype": "f64"},
        }
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
