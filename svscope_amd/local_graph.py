"""localGraph_npz on MI355X: the batched caller of the per-window path.

Mirrors /root/reference/src/SVscope.py:185-239 (localGraph_npz): read every
``*npz*`` bundle in ``savedir`` (``DatSet`` rows [sequenceList, ReadIDs,
flank_5, flank_3, TDRecord], SomTDDetector_AimDatFetch.py:118,160-183), run
TDscope_npz on each window, write ``<T>.vs.<N>.TandemRepeat.Raw.bed`` (one
"\\t".join(str(field)) line per window, :175) and sort it like
``sort -k1,1 -k2,2n`` (:236; C-locale byte order, whole-line tie-break).

Differences, all deliberate:
  * windows run in GPU batches (DecisionBatch) instead of a 6-process Pool;
  * ``--Continue`` skips windows whose first three fields are already in the
    output (the reference compares full records against 3-field keys and so
    never skips);
  * multi-GPU: one process per GPU (torch.distributed, backend "nccl" = RCCL);
    windows are dealt to ranks longest-first by estimated cost N*L^2, each rank
    runs its shard on its own GPU, and rank 0 receives every rank's packed
    records with one RCCL all_gather over xGMI.  No other collective exists:
    windows are independent (per-window RNG reseed).
"""
import argparse
import logging
import os
import re
import time

import numpy as np

from .som_td_detector import TDscope_npz_batch

log = logging.getLogger("svscope_amd")


def load_bundles(savedir):
    rows = []
    for name in sorted(os.listdir(savedir)):
        if re.search("npz", name):
            dat = np.load(os.path.join(savedir, name), allow_pickle=True)["DatSet"]
            rows.extend(list(dat))
    return rows


def window_cost(row):
    seqs = row[0]
    n = max(1, len(seqs) - 1)
    mean_len = (sum(len(s) for s in seqs) / max(1, len(seqs)))
    return n * mean_len * mean_len


def shard_lpt(rows, world):
    """Longest-processing-time-first assignment of windows to ranks."""
    order = sorted(range(len(rows)), key=lambda i: -window_cost(rows[i]))
    load = [0.0] * world
    owner = [0] * len(rows)
    for i in order:
        r = min(range(world), key=lambda k: (load[k], k))
        owner[i] = r
        load[r] += window_cost(rows[i])
    return owner


def record_line(rec):
    return "\t".join(str(x) for x in rec)


def sort_lines(lines):
    """sort -k1,1 -k2,2n with C-locale collation and whole-line last resort."""
    def key(line):
        f = line.split("\t")
        m = re.match(r"\s*([+-]?\d+)", f[1]) if len(f) > 1 else None
        return (f[0].encode(), int(m.group(1)) if m else 0, line.encode())
    return sorted(lines, key=key)


def run_windows(rows, batch_size=512, context=None, stats=None):
    out = []
    for s in range(0, len(rows), batch_size):
        out.extend(TDscope_npz_batch(rows[s:s + batch_size], context=context, stats=stats))
    return out


def gather_lines(lines, device):
    """RCCL all_gather of every rank's packed record lines (rank 0 keeps them)."""
    import torch
    import torch.distributed as dist
    payload = "\n".join(lines).encode()
    n = torch.tensor([len(payload)], dtype=torch.int64, device=device)
    sizes = [torch.zeros_like(n) for _ in range(dist.get_world_size())]
    dist.all_gather(sizes, n)
    cap = int(max(s.item() for s in sizes))
    buf = torch.zeros(max(cap, 1), dtype=torch.uint8, device=device)
    if payload:
        buf[:len(payload)] = torch.frombuffer(bytearray(payload), dtype=torch.uint8).to(device)
    bufs = [torch.zeros_like(buf) for _ in sizes]
    dist.all_gather(bufs, buf)
    out = []
    for s, b in zip(sizes, bufs):
        k = int(s.item())
        if k:
            out.extend(bytes(b[:k].cpu().numpy()).decode().split("\n"))
    return out


def localGraph_npz(args):
    t0 = time.time()
    tsid = args.TSampleID.split(",")
    nsid = args.NSampleID.split(",")
    rawoutput = "%s.vs.%s.TandemRepeat.Raw.bed" % ("-".join(tsid), "-".join(nsid))
    path = os.path.join(args.savedir, rawoutput)
    rows = load_bundles(args.savedir)
    finished = set()
    if getattr(args, "Continue", False) and os.path.exists(path):
        with open(path) as fh:
            finished = {"\t".join(x.strip().split("\t")[0:3]) for x in fh if x.strip()}
    rows = [r for r in rows if "\t".join(r[4].strip().split("\t")[0:3]) not in finished]

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        import torch
        import torch.distributed as dist
        local = int(os.environ.get("LOCAL_RANK", "0"))
        # RCCL between GPUs; gloo only for CPU rehearsals of the plumbing (the
        # windows themselves still need the HIP engine)
        gpu = torch.cuda.is_available()
        if gpu:
            torch.cuda.set_device(local)
            os.environ.setdefault("SVS_DEVICE", str(local))
        if not dist.is_initialized():
            dist.init_process_group("nccl" if gpu else "gloo")
        owner = shard_lpt(rows, world)
        mine = [r for r, o in zip(rows, owner) if o == rank]
        lines = [record_line(x) for x in run_windows(mine, args.batch)]
        lines = gather_lines(lines, torch.device("cuda", local) if gpu else torch.device("cpu"))
    else:
        lines = [record_line(x) for x in run_windows(rows, args.batch)]
    if rank == 0:
        mode = "a" if finished else "w"
        with open(path, mode) as fh:
            for line in lines:
                fh.write(line + "\n")
        with open(path) as fh:
            allines = [x.rstrip("\n") for x in fh if x.strip()]
        with open(path, "w") as fh:
            for line in sort_lines(allines):
                fh.write(line + "\n")
        log.info("Local Graph : work finished with %s hour", (time.time() - t0) / 3600)
    return path


def main(argv=None):
    ap = argparse.ArgumentParser(description="SVScope localGraph_npz on MI355X")
    ap.add_argument("-t", "--TSampleID", required=True)
    ap.add_argument("-n", "--NSampleID", required=True)
    ap.add_argument("-s", "--savedir", required=True)
    ap.add_argument("-p", "--thread", default="6")
    ap.add_argument("-o", "--offset", type=int, default=50)
    ap.add_argument("-q", "--mapQ", type=int, default=5)
    ap.add_argument("-C", "--Continue", action="store_true")
    ap.add_argument("--batch", type=int, default=512, help="windows per GPU batch")
    args = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s - %(levelname)s - %(message)s")
    print(localGraph_npz(args))


if __name__ == "__main__":
    main()
