#!/usr/bin/env python3
"""Benchmark of the SVScope localGraph hot path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--depth D]

Workload: BASELINE.json configs[2] ("config 3"): candidate windows of 64 reads
x 3 kb, synthetic (SURVEY.md §8(d) generator), run end to end through the
localGraph per-window path (window MSA POA -> feature selection -> EM over
K=1..9 -> per-cluster consensus POA -> 10-field record).

One step = one batch of B windows (default 512) submitted to the engine's
streaming decision session.  K steps = K*B windows (default 20 x 512 = 10,240,
i.e. config 3's 10,000 windows) are all submitted and completed inside the
timed region; the session keeps up to D batches in flight (continuous
batching: batch b+1's window MSAs fill the GPU while batch b finishes), the
way localGraph_npz streams its windows.  Warmup steps run W batches of a
separate, reused set of B windows through the same session before timing.

The timed region ends with the sorted Raw.bed lines (local_graph.record_line
and sort_lines, SVscope.py:171-180, 236).

For --gpus N > 1 the script re-launches itself under torch.distributed.run
(one process per GPU, before anything touches a GPU).  The N ranks share one
global set of N*K*B windows, dealt by LPT over their cost N*L^2
(local_graph.lpt_owner, as localGraph_npz deals its windows; the costs are
exchanged through the rendezvous store before any GPU call).  Timed on every
rank: its windows through its own session, then one RCCL gather of every
rank's record lines to rank 0 (local_graph.gather_payloads) and rank 0's sort
(local_graph.sort_payloads).
Time = max over ranks, value = N*K*B / that time (weak scaling: K*B windows
per GPU on average).

roofline: the dominant kernel is the POA DP (poa_strip_kernel).  achieved /
frac = algorithmic bytes (20 B per evaluated DP cell: the int32 H,E,F,O,Q
planes of convex NW) of the timed DP launches over the device
time during which at least one of them ran (the union of their HIP-event
intervals on the two task groups' DP streams; tools/rocprof_timed.py restates
it from a rocprofv3 kernel trace); per_launch divides by the summed launch
durations instead, and frac_over_wall by the timed region.  traffic = measured
HBM bytes per evaluated cell from the committed rocprofv3 PMC summary
(profiles/pmc_poa_traffic.json) x cells per launch, else null.

cpu_baseline: the CPU oracle (C++ spoa restatement standing in for pyspoa, the
numpy EM restatement of ReadsCluster.py, the literal Decision) on a bounded
sample of the same windows, timed before the GPU is touched, in the two modes
of SURVEY.md §8(d): as shipped (min(6, cores) worker processes,
SVscope.py:158-161) and all cores of this job's CPU share, BLAS threads 1.
"""
import argparse
import json
import multiprocessing as mp
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "candidate-windows/sec (64 reads × 3 kb) localGraph, 1/2/4/8 MI355X; % HBM roofline"
HBM_PEAK_GBS = 8000.0
FP64_MATRIX_PEAK_TFLOPS = 78.6  # MI355X dense FP64 matrix peak (the EM's dtype)
BYTES_PER_CELL = 20
GOLDEN_DIGESTS = os.path.join(ROOT, "tests", "golden", "bench_config3_digests.json")
N_READS, REF_LEN = 64, 3000
WARMUP_ID_BASE = 1 << 30  # warmup windows never share a seed with timed ones


def _gen(ws):
    from svscope_amd import synth
    return [synth.make_window(w, N_READS, REF_LEN) for w in ws]


def _costs(ws):
    from svscope_amd import synth
    from svscope_amd.local_graph import cost_of_lengths
    return [cost_of_lengths(synth.window_lengths(w, N_READS, REF_LEN)) for w in ws]


def window_costs(ids, procs):
    """LPT costs of windows ids (local_graph.window_cost of each row) from
    their lengths alone (synth.window_lengths), in `procs` processes."""
    if procs <= 1 or len(ids) < 2:
        return _costs(ids)
    chunks = [ids[i::procs] for i in range(procs)]
    pool = mp.get_context("fork").Pool(procs)
    try:
        parts = pool.map(_costs, chunks)
    finally:
        pool.close()
        pool.join()
    out = [0.0] * len(ids)
    for i, part in enumerate(parts):
        out[i::procs] = part
    return out


def generate(ids, procs):
    if procs <= 1 or len(ids) < 2:
        return _gen(ids)
    chunks = [ids[i::procs] for i in range(procs)]
    # close + join, not the context manager: its exit terminates the workers
    # (SIGTERM), which a profiler's signal handler reports as an abort
    pool = mp.get_context("fork").Pool(procs)
    try:
        parts = pool.map(_gen, chunks)
    finally:
        pool.close()
        pool.join()
    by_id = {}
    for chunk, part in zip(chunks, parts):
        for w, row in zip(chunk, part):
            by_id[w] = row
    return [by_id[w] for w in ids]


def host_cores():
    """CPUs this job may use: its affinity mask, capped by the box's CPU share
    (OMP_NUM_THREADS is set to the share on the GPU boxes)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    share = os.environ.get("OMP_NUM_THREADS")
    if share and share.isdigit() and int(share) > 0:
        n = min(n, int(share))
    return max(1, n)


def _baseline_init():
    from threadpoolctl import threadpool_limits
    threadpool_limits(1)  # BLAS threads = 1 per worker


def _oracle_window(row):
    import numpy as np
    from oracle import decision_oracle
    return decision_oracle.tdscope_npz(row[4], row[0], np.asarray(row[1]), row[2], row[3])


def _time_pool(rows, workers):
    t = time.time()
    pool = mp.get_context("fork").Pool(workers, initializer=_baseline_init)
    try:
        pool.map(_oracle_window, rows, chunksize=1)
    finally:
        pool.close()
        pool.join()
    return time.time() - t


def cpu_baseline(rows, cores):
    """Both §8(d) modes, one window per worker each, before any GPU call."""
    from oracle import spoa_oracle
    spoa_oracle._load()  # build/load the C++ oracle before timing
    shipped = min(6, cores)
    modes = {}
    for name, workers in (("as_shipped", shipped), ("all_cores", cores)):
        sample = rows[:workers]
        wall = _time_pool(sample, workers)
        modes[name] = {"value": round(len(sample) / wall, 5), "workers": workers, "windows": len(sample),
                       "wall_s": round(wall, 2)}
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    best = modes["all_cores"]
    return {"value": best["value"], "unit": "windows/s", "cores": best["workers"], "kind": "port",
            "sample": (f"one config-3 window (64 reads x 3 kb) per worker process; as shipped "
                       f"{modes['as_shipped']['workers']} workers (SVscope.py:158-161), all cores "
                       f"{best['workers']} workers (this job's CPU share); BLAS threads 1; POA is a proxy: "
                       f"the C++ spoa-NW-convex restatement (pyspoa is not installed), numpy EM, literal Decision"),
            "modes": modes, "cpu_model": model, "nproc": os.cpu_count()}


def cpu_baseline_process():
    """cpu_baseline in a child Python process (same windows: ids 0 .. cores-1),
    started before this process touches the GPU, so that the bench's own
    process carries none of the baseline's imports, oracle library or fork
    pools.  (It was first taken for the cause of the slow final-drain runs,
    DESIGN §7 item 2; those also occur with --cpu-sample 0, profiles/r06_eb.)"""
    import tempfile
    fd, path = tempfile.mkstemp(suffix=".json")
    os.close(fd)
    try:
        subprocess.run([sys.executable, os.path.abspath(__file__), "--cpu-baseline-json", path], check=True)
        with open(path) as fh:
            return json.load(fh)
    finally:
        os.unlink(path)


def pmc_traffic_per_cell():
    """Measured HBM bytes per evaluated DP cell of the POA kernel from the
    committed rocprofv3 PMC summary (FETCH_SIZE and WRITE_SIZE passes), or None."""
    path = os.path.join(ROOT, "profiles", "pmc_poa_traffic.json")
    if not os.path.exists(path):
        return None
    try:
        return float(json.load(open(path))["hbm_bytes_per_cell"])
    except Exception:
        return None


def record_digests(lines):
    """SHA-256 of each timed record's Raw.bed line (local_graph.record_line,
    SVscope.py:171-180) for the windows the committed CPU-oracle fixture covers
    (tests/golden/bench_config3_digests.json: window ids 0..255, and every 40th
    id after them up to 10,239, so that every timed step of rank 0's N = 1 run
    is checked), found among the sorted lines by their window's chrom / start /
    end (synth.window_key), and whether they all match it.  None when the
    fixture covers none of them."""
    import hashlib
    from svscope_amd import synth
    if not os.path.exists(GOLDEN_DIGESTS):
        return None
    gold = json.load(open(GOLDEN_DIGESTS))
    by_key = {"\t".join(x.split("\t")[0:3]): x for x in lines}

    def digest(w):
        line = by_key.get(synth.window_key(w, REF_LEN))
        return hashlib.sha256(line.encode()).hexdigest() if line is not None else None
    n = 0
    while n < len(gold["digests"]) and synth.window_key(n, REF_LEN) in by_key:
        n += 1
    if n == 0:
        return None
    got = [digest(k) for k in range(n)]
    bad = [k for k in range(n) if got[k] != gold["digests"][k]]
    out = {"windows": n, "digest": hashlib.sha256("\n".join(got).encode()).hexdigest(),
           "oracle_digest": gold["all"] if n == len(gold["digests"]) else None,
           "match": not bad, "mismatched_windows": bad[:16]}
    sp = [(w, d) for w, d in zip(gold.get("sparse_ids", []), gold.get("sparse_digests", []))
          if synth.window_key(w, REF_LEN) in by_key]
    if sp:
        sbad = [w for w, d in sp if digest(w) != d]
        out["sparse"] = {"windows": len(sp), "first_id": sp[0][0], "last_id": sp[-1][0], "match": not sbad,
                         "mismatched_windows": sbad[:16]}
        out["match"] = out["match"] and not sbad
        out["windows_checked"] = n + len(sp)
    return out


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv):
    """Runs this script as n ranks under torch.distributed.run (a child process:
    nothing here has touched the GPU) and returns its exit code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + argv
    return subprocess.call(cmd)


# levels, not counters: the timed region reports them as they are at its end
LEVEL_STATS = {"dgraph_peak_bytes", "dgraph_reserved_bytes"}


def diff_stats(a, b):
    out = {}
    for k, v in b.items():
        if isinstance(v, dict):
            out[k] = diff_stats(a.get(k, {}), v)
        else:
            out[k] = v if k in LEVEL_STATS else v - a.get(k, 0)
    return out


def run_steps(session, batches, depth):
    """Submits every batch, at most `depth` in flight; returns the records."""
    from collections import deque
    tickets, out = deque(), []
    for b in batches:
        tickets.append(session.submit(b))
        if len(tickets) >= depth:
            out.extend(session.wait(tickets.popleft()))
    while tickets:
        out.extend(session.wait(tickets.popleft()))
    return out


def deal_global(world, rank, K, B, gen_procs, store):
    """N > 1: one global set of world*K*B window ids dealt to the ranks by
    local_graph.lpt_owner (LPT over N*L^2, what localGraph_npz does with its
    windows, local_graph.shard_lpt).  Each rank computes the costs of every
    world-th id (from the windows' lengths alone, synth.window_lengths), the
    ranks exchange them through the rendezvous store (no GPU is touched yet),
    every rank computes the same deal, and each rank then generates the
    windows it owns.  Returns this rank's owned ids (ascending), their rows,
    and every rank's window count and cost."""
    import numpy as np
    from svscope_amd.local_graph import lpt_owner
    n_all = world * K * B
    stripe = list(range(rank, n_all, world))
    mine = np.array(window_costs(stripe, gen_procs), dtype=np.float64)
    store.set(f"cost{rank}", mine.tobytes())
    costs = np.empty(n_all, dtype=np.float64)
    for r in range(world):
        costs[r::world] = np.frombuffer(store.get(f"cost{r}"), dtype=np.float64)
    owner = lpt_owner(costs.tolist(), world)
    ids = [w for w in range(n_all) if owner[w] == rank]
    out = generate(ids, gen_procs)
    per_n = [0] * world
    per_cost = [0.0] * world
    for w, r in enumerate(owner):
        per_n[r] += 1
        per_cost[r] += float(costs[w])
    return ids, out, per_n, per_cost


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=int(os.environ.get("SVS_BENCH_BATCH", "512")))
    # 14 batches in flight, as localGraph_npz streams (local_graph.iter_batches):
    # 7168 windows keep both task groups at their 2048 active POA tasks
    # (driver-shape A/B, profiles/r04_ab4..r04_ab6: 4 batches / 1024 tasks 273.7,
    # 8 / 1536 302.5-304.6, 10 / 1792 301.4-311.1 windows/s; with 2048 tasks,
    # profiles/r04_i2, r04_i3: 10 batches 351.2, 12 354.5-357.2, 14
    # 359.2-360.6, 16 358.6, 20 358.4)
    ap.add_argument("--depth", type=int, default=int(os.environ.get("SVS_BENCH_DEPTH", "14")),
                    help="batches in flight in the streaming session")
    ap.add_argument("--cpu-sample", type=int, default=-1, help="CPU baseline: -1 both modes, 0 off")
    ap.add_argument("--gen-procs", type=int, default=0, help="window generator processes (0: all host cores)")
    ap.add_argument("--probe-env", default="", help=argparse.SUPPRESS)  # launcher test: record rank env, exit
    ap.add_argument("--cpu-baseline-json", default="", help=argparse.SUPPRESS)  # the baseline's own process
    args = ap.parse_args()

    if args.cpu_baseline_json:
        # the CPU baseline in a process of its own (see cpu_baseline_process)
        cores = host_cores()
        with open(args.cpu_baseline_json, "w") as fh:
            json.dump(cpu_baseline(generate(list(range(cores)), cores), cores), fh)
        return

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.probe_env:
        with open(os.path.join(args.probe_env, f"rank{rank}.json"), "w") as fh:
            json.dump({k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR")}, fh)
        return
    if world != args.gpus and rank == 0:
        print(f"[bench] note: WORLD_SIZE={world} overrides --gpus {args.gpus}", file=sys.stderr)

    # Everything that forks (window generation, the CPU baseline) runs before
    # this process touches the GPU.
    B, K, W = max(1, args.batch), max(1, args.steps), max(0, args.warmup)
    cores = host_cores()
    gen_procs = args.gen_procs or max(1, cores // max(1, world) if world > 1 else cores)
    t_gen = time.time()
    store = None
    deal = None
    if world > 1:
        # the rendezvous store (torchrun's agent store, or rank 0's): the cost
        # exchange of the deal, then the process group below
        import torch.distributed as dist
        from torch.distributed import PrefixStore
        store = next(dist.rendezvous("env://", rank, world))[0]
        timed_ids, rows, per_n, per_cost = deal_global(world, rank, K, B, gen_procs,
                                                       PrefixStore("svs_bench_deal", store))
        deal = {"windows": per_n, "lpt_cost": per_cost}
    else:
        timed_ids = list(range(K * B))
        rows = generate(timed_ids, gen_procs)
    warm = generate(list(range(WARMUP_ID_BASE + rank * B, WARMUP_ID_BASE + (rank + 1) * B)), gen_procs) if W else []
    # bundle rows [sequenceList, ReadIDs, flank_5, flank_3, TDRecord] -> the
    # TDscope_npz arguments, as localGraph_npz passes them (SVscope.py:212-217)
    from svscope_amd.local_graph import _window
    batches = [[_window(r) for r in rows[s:s + B]] for s in range(0, len(rows), B)]
    warm = [_window(r) for r in warm]
    gen_s = time.time() - t_gen

    cpu = None
    if args.cpu_sample != 0 and world == 1 and rank == 0:  # the CPU baseline is an N=1 figure
        cpu = cpu_baseline_process()

    dist = None
    device = None
    if world > 1:
        # this rank's CPU slice and engine pool size (svscope_amd/hostcpu.py),
        # before the library creates its context
        from svscope_amd import hostcpu
        hostcpu.apply(local, int(os.environ.get("LOCAL_WORLD_SIZE", world)))
        import torch
        import torch.distributed as dist
        from svscope_amd.local_graph import rank_device
        # RCCL over the node's GPUs, one per rank; SVS_DIST_BACKEND=gloo with
        # SVS_DEVICE=d rehearses the N > 1 path with every rank on GPU d
        backend = os.environ.get("SVS_DIST_BACKEND", "nccl")
        local = rank_device(backend, local, os.environ)
        torch.cuda.set_device(local)
        os.environ["SVS_DEVICE"] = str(local)
        if backend == "nccl":
            device = torch.device("cuda", local)
            dist.init_process_group("nccl", store=store, rank=rank, world_size=world, device_id=device)
        else:
            device = torch.device("cpu")
            dist.init_process_group(backend, store=store, rank=rank, world_size=world)

    from svscope_amd import _abi
    from svscope_amd.decision_maker import DecisionSession
    from svscope_amd.local_graph import gather_payloads, record_line, sort_lines, sort_payloads
    ctx = _abi.default_context(local if world > 1 else None)
    session = DecisionSession(ctx)

    t_warm = time.time()
    if W:
        run_steps(session, [warm] * W, args.depth)
    warm_s = time.time() - t_warm
    st0 = session.stats()

    # Timed: every owned window through the session, the Raw.bed lines, then
    # (N > 1) rank 0 receives every rank's lines with one RCCL gather
    # (local_graph.gather_payloads, after an 8-B all_gather of the sizes), and
    # rank 0 sorts them like sort -k1,1 -k2,2n (SVscope.py:158-180, 236).
    if dist is not None:
        import torch
        dist.barrier()
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    recs = run_steps(session, batches, args.depth)
    lines = [record_line(r) for r in recs]
    t_own = time.perf_counter() - t0
    if dist is not None:
        # every rank's record bytes to rank 0, which sorts them without a
        # Python string per record (local_graph.sort_payloads)
        payloads = gather_payloads("\n".join(lines).encode(), device)
        out = sort_payloads(payloads) if rank == 0 else b""
    else:
        out = sort_lines(lines)
    if dist is not None:
        dist.barrier()
        torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    st = diff_stats(st0, session.stats())
    session.close()
    n_em = sum(1 for r in recs if str(r[-1]).endswith("|EMOutput"))
    assert len(recs) == len(timed_ids), (len(recs), len(timed_ids))
    if rank == 0:
        out_lines = out if dist is None else out.decode().split("\n")
        assert len(out_lines) == K * B * world, (len(out_lines), K * B * world)
    ranks = None
    if dist is not None:
        # every rank's own figures (SCALE shows LPT / box imbalance), then
        # time = the max over ranks
        gdev = device if dist.get_backend() == "nccl" else "cpu"
        mine = torch.tensor([elapsed, t_own, float(len(recs))], dtype=torch.float64, device=gdev)
        every = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(every, mine)
        per = [x.tolist() for x in every]
        elapsed = max(p[0] for p in per)
        own = [p[1] for p in per]
        ranks = {"elapsed_s": [round(p[0], 3) for p in per], "own_windows_s": [round(x, 3) for x in own],
                 "windows": [int(p[2]) for p in per], "lpt_windows": deal["windows"],
                 "lpt_cost": [round(c / 1e9, 3) for c in deal["lpt_cost"]], "lpt_cost_unit": "G (reads x len^2)",
                 "own_max_over_mean": round(max(own) / (sum(own) / len(own)), 4),
                 "gather_and_sort_s": round(elapsed - max(own), 3),
                 "note": "own_windows_s: a rank's windows through its session to their record lines; "
                         "elapsed_s adds the RCCL gather of every rank's lines to rank 0 and rank 0's sort"}

    poa = st["poa"]
    cells, cells_done = poa["dp_cells"], poa["cells_computed"]
    kms, launches = poa["kernel_ms"], poa["launches"]
    algo_bytes = cells_done * BYTES_PER_CELL
    per_launch = algo_bytes / (kms * 1e-3) / 1e9 if kms > 0 else 0.0
    busy_ms = poa.get("kernel_busy_ms", 0.0)
    busy_achieved = algo_bytes / (busy_ms * 1e-3) / 1e9 if busy_ms > 0 else 0.0
    total_windows = B * K * world

    em_flops = st.get("em_flops", 0.0)
    em_s = st["em_kernel_ms"] / 1e3
    em_tflops = em_flops / em_s / 1e12 if em_s > 0 else 0.0
    if rank == 0:
        value = total_windows / elapsed
        digests = record_digests(out_lines)
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
            "config": {"workload": f"config3: {K * B} candidate windows per GPU (64 reads x 3 kb), {B} per step, "
                                   f"localGraph end to end (MSA POA + features + EM K=1..9 + consensus POA) "
                                   f"to the sorted Raw.bed lines"
                                   + (f"; {K * B * world} windows dealt to {world} ranks by LPT, records "
                                      f"gathered to rank 0 over {dist.get_backend()}" if world > 1 else ""),
                       "windows_per_step_per_gpu": B, "windows_per_gpu": K * B, "reads_per_window": N_READS,
                       "ref_len": REF_LEN, "batches_in_flight": args.depth,
                       "parallelism": f"window shards x{world}"},
            # frac: the DP kernel's algorithmic bytes (20 B per evaluated cell,
            # SURVEY.md §8(d)) over the device time during which at least one of
            # the timed DP launches ran (the union of their HIP-event intervals,
            # kernel_busy_ms; tools/rocprof_timed.py restates it from a
            # rocprofv3 kernel trace).  The two task groups' launches overlap on
            # their DP streams, so per-launch durations count the shared time
            # twice; that figure is per_launch below.
            "roofline": {"bound": "hbm", "kernel": "poa_strip_kernel",
                         "achieved": round(busy_achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(busy_achieved / HBM_PEAK_GBS, 5),
                         "basis": "algorithmic bytes of the timed DP launches / union of their intervals",
                         "busy_ms": round(busy_ms, 2),
                         "traffic": traffic, "traffic_basis": "HBM bytes per DP launch (PMC bytes per evaluated "
                                                              "cell, profiles/pmc_poa_traffic.json, x cells per launch)",
                         "algorithmic_bytes_per_launch": int(algo_bytes / max(1, launches)),
                         # the same bytes over the whole timed region (rank 0's GPU)
                         "frac_over_wall": round(algo_bytes / elapsed / 1e9 / HBM_PEAK_GBS, 5),
                         "per_launch": {"achieved": round(per_launch, 2),
                                        "frac": round(per_launch / HBM_PEAK_GBS, 5),
                                        "mean_launch_ms": round(kms / max(1, launches), 4),
                                        "launch_ms_over_busy_ms": round(kms / busy_ms, 4) if busy_ms else None},
                         # SURVEY.md §8(d) prices Σcells over every DP cell of spoa's full
                         # matrix (its "50 % needs ~2e11 cells/s, ~100 windows/s");
                         # frac above counts only the cells the pruned kernel evaluates
                         "all_dp_cells": {"achieved": round(cells * BYTES_PER_CELL / (kms * 1e-3) / 1e9, 2)
                                          if kms else None,
                                          "frac": round(cells * BYTES_PER_CELL / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)
                                          if kms else None,
                                          "note": "every DP cell of the full matrix; above 1 because exact "
                                                  "pruning skips most cells, so not an HBM-traffic figure"}},
            "cpu_baseline": cpu,
            "oracle_check": digests,
            "ranks": ranks,
            "breakdown": {"poa_cells": cells, "poa_cells_computed": cells_done,
                          "prune_retries": poa["prune_retries"],
                          # HIP events between the kernels on each group's fold stream
                          # (device-resident graphs), timed steps only; they run beside
                          # the other group's DP kernel
                          "fold_kernel_ms": {"poa_fold_update_kernel": round(poa["fold_update_ms"], 1),
                                             "poa_fold_sort_kernel": round(poa["fold_sort_ms"], 1),
                                             "poa_fold_final_kernel": round(poa["fold_final_ms"], 1),
                                             "poa_dgraph_prep_kernel": round(poa["fold_prep_ms"], 1)},
                          # the group's next launch waits for this after each DP launch
                          "dp_end_to_launch_done_ms": round(poa.get("dp_to_done_ms", 0.0), 1),
                          "poa_table_exports": poa.get("prep_jobs", 0),
                          "poa_kernel_ms": round(kms, 2), "poa_launches": launches,
                          "poa_deferred_tasks": poa.get("deferred_tasks", 0),
                          "dgraph_peak_gb": round(poa.get("dgraph_peak_bytes", 0) / 2**30, 2),
                          "dgraph_reserved_gb": round(poa.get("dgraph_reserved_bytes", 0) / 2**30, 2),
                          "gcups": round(cells_done / (kms * 1e-3) / 1e9, 3) if kms else None,
                          "gcups_full_matrix_equivalent": round(cells / (kms * 1e-3) / 1e9, 3) if kms else None,
                          "host_graph_ms": round(poa["host_graph_ms"], 1),
                          "host_wait_for_gpu_ms": round(poa["gpu_wait_ms"], 1),
                          "h2d_bytes": poa["h2d_bytes"], "d2h_bytes": poa["d2h_bytes"],
                          "em_output_windows": n_em,
                          "em_kernel_s": round(st["em_kernel_ms"] / 1e3, 3),
                          # EM roofline is the FP64 matrix peak;
                          # dense-equivalent FLOPs = sum_K 41 x 2 N (5 nf) K per window
                          "em_roofline": {"bound": "mfma", "dense_equiv_flops": em_flops,
                                          "achieved": round(em_tflops, 3), "peak": FP64_MATRIX_PEAK_TFLOPS,
                                          "unit": "TFLOP/s", "frac": round(em_tflops / FP64_MATRIX_PEAK_TFLOPS, 5)},
                          "em_wall_s": round(st["em_wall_ms"] / 1e3, 3),
                          "em_launches": st["em_launches"], "em_windows": st["em_windows"],
                          "em_reruns_in_order": st["em_reruns"],
                          "consensus_tasks": st["consensus_tasks"],
                          "features_s": round(st["features_ms"] / 1e3, 3),
                          "labelling_s": round(st["labelling_ms"] / 1e3, 3),
                          "generate_s": round(gen_s, 1), "warmup_s": round(warm_s, 1),
                          "em_dtype": "f64"},
        }
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
