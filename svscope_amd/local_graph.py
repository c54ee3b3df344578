"""localGraph_npz on MI355X: the batched caller of the per-window path.

Mirrors /root/reference/src/SVscope.py:185-239 (localGraph_npz): read every
``*npz*`` bundle in ``savedir`` (``DatSet`` rows [sequenceList, ReadIDs,
flank_5, flank_3, TDRecord], SomTDDetector_AimDatFetch.py:118,160-183), run
TDscope_npz on each window, write ``<T>.vs.<N>.TandemRepeat.Raw.bed`` (one
"\\t".join(str(field)) line per window, :175) and sort it like
``sort -k1,1 -k2,2n`` (:236; C-locale byte order, whole-line tie-break).

Differences, all deliberate:
  * windows stream through one DecisionSession in GPU batches instead of a
    6-process Pool; each batch's records are appended and flushed as soon as
    the batch completes (the reference flushes per record), so --Continue
    resumes after a crash (per-rank journals ``<out>.part<rank>`` on N > 1,
    folded into the output by rank 0 on the next --Continue run);
  * ``--Continue`` skips windows whose first three fields are already in the
    output (the reference compares full records against 3-field keys and so
    never skips);
  * multi-GPU: one process per GPU (torch.distributed, backend "nccl" = RCCL);
    windows are dealt to ranks longest-first by estimated cost N*L^2, each rank
    runs its shard on its own GPU, and rank 0 receives every rank's packed
    records with one RCCL gather over xGMI (after an 8-byte all_gather of
    the byte counts).  No other collective exists:
    windows are independent (per-window RNG reseed).
"""
import argparse
import logging
import os
import re
import time

import numpy as np


log = logging.getLogger("svscope_amd")


def load_bundles(savedir):
    rows = []
    for name in sorted(os.listdir(savedir)):
        if re.search("npz", name):
            dat = np.load(os.path.join(savedir, name), allow_pickle=True)["DatSet"]
            rows.extend(list(dat))
    return rows


def window_cost(row):
    return cost_of_lengths([len(s) for s in row[0]])


def cost_of_lengths(lens):
    """A window's LPT cost from its sequence lengths (reference row first):
    reads x mean length^2."""
    n = max(1, len(lens) - 1)
    mean_len = sum(lens) / max(1, len(lens))
    return n * mean_len * mean_len


def shard_lpt(rows, world):
    """Longest-processing-time-first assignment of windows to ranks."""
    return lpt_owner([window_cost(r) for r in rows], world)


def lpt_owner(costs, world):
    """LPT over window costs: the costliest window first, each to the least
    loaded rank (lowest rank on ties); returns each window's rank.  Every
    rank computes the same deal from the same costs (bench.py deals its
    global window set this way from costs exchanged before the GPU starts)."""
    import heapq
    order = sorted(range(len(costs)), key=lambda i: (-costs[i], i))
    heap = [(0.0, k) for k in range(world)]
    owner = [0] * len(costs)
    for i in order:
        load, r = heapq.heappop(heap)
        owner[i] = r
        heapq.heappush(heap, (load + costs[i], r))
    return owner


def record_line(rec):
    return "\t".join(str(x) for x in rec)


def sort_lines(lines):
    """sort -k1,1 -k2,2n with C-locale collation and whole-line last resort.
    (Python compares str by code point, which is UTF-8 byte order, i.e. the C
    locale's; only the first two fields are split off.)"""
    def key(line):
        f = line.split("\t", 2)
        if len(f) < 2:
            return (f[0], 0, line)
        v = f[1]
        if v.isdigit():
            return (f[0], int(v), line)
        m = re.match(r"\s*([+-]?\d+)", v)
        return (f[0], int(m.group(1)) if m else 0, line)
    return sorted(lines, key=key)


def _window(r):
    """bundle row [sequenceList, ReadIDs, flank_5, flank_3, TDRecord] -> Decision arguments"""
    return (r[4], list(r[0]), np.asarray(r[1]), r[2], r[3])


def iter_batches(rows, batch_size=512, context=None, depth=14):
    """Yields the records of each batch of ``rows``, in order, streamed through
    one DecisionSession with up to ``depth`` batches in flight (the engine's
    scheduler never drains between batches; 14 x 512 windows keep both task
    groups at their 2048 active POA tasks, bench.py --depth).  A window past an engine limit
    (decision_maker.WindowFailed) yields None in its place; the others run on,
    and once every batch is done a WindowFailed names all such windows (row
    indices into ``rows``)."""
    from collections import deque
    from .decision_maker import DecisionSession, WindowFailed
    if not rows:
        return
    failed = {}

    def take(session, ticket, base):
        try:
            return session.wait(ticket)
        except WindowFailed as e:
            failed.update({base + w: why for w, why in e.failed.items()})
            return e.records

    with DecisionSession(context) as session:
        tickets = deque()
        for k in range(0, len(rows), batch_size):
            tickets.append((session.submit([_window(r) for r in rows[k:k + batch_size]]), k))
            if len(tickets) >= depth:
                yield take(session, *tickets.popleft())
        while tickets:
            yield take(session, *tickets.popleft())
    if failed:
        raise WindowFailed(failed, None)


def run_windows(rows, batch_size=512, context=None):
    """Records of ``rows`` in order; a WindowFailed carries them (None for the
    failed windows) in ``records``."""
    from .decision_maker import WindowFailed
    out = []
    try:
        for recs in iter_batches(rows, batch_size, context):
            out.extend(recs)
    except WindowFailed as e:
        e.records = out
        raise
    return out


def write_journal(path, mode, rows, batch_size, failed=None):
    """Runs the windows and appends each batch's records to ``path`` as soon as
    the batch completes, flushed (the reference writes and flushes every
    record as it arrives, SVscope.py:227-233, which is what makes --Continue
    resume after a crash).  Returns the record lines.  Windows past an engine
    limit are left out of the journal; with ``failed`` (a dict) given, their
    TDRecord keys and reasons go there and the call returns normally, so that
    the caller still gathers and sorts every other record."""
    from .decision_maker import WindowFailed
    lines = []
    with open(path, mode) as fh:
        try:
            for recs in iter_batches(rows, batch_size):
                chunk = [record_line(x) for x in recs if x is not None]
                fh.write("".join(line + "\n" for line in chunk))
                fh.flush()
                lines.extend(chunk)
        except WindowFailed as e:
            if failed is None:
                raise
            failed.update({window_key(rows[i]): why for i, why in e.failed.items()})
    return lines


def window_key(row):
    """chrom, start, end of a bundle row's TDRecord (the --Continue key)."""
    return "\t".join(row[4].strip().split("\t")[0:3])


def _report_failed(failed, rank):
    """After the output is complete: every window past an engine limit, named
    by its TDRecord key, in one WindowFailed (each rank its own)."""
    from .decision_maker import WindowFailed
    if failed:
        for key, why in sorted(failed.items()):
            log.error("rank %d: window %s not written: %s", rank, key.replace("\t", ":"), why)
        raise WindowFailed(failed, None)


def part_path(path, rank):
    return "%s.part%d" % (path, rank)


def merge_parts(path):
    """Folds the per-rank journals of an interrupted multi-GPU run into the
    output file (rank 0, before any window runs)."""
    d, base = os.path.split(path)
    parts = sorted(x for x in os.listdir(d or ".") if re.fullmatch(re.escape(base) + r"\.part\d+", x))
    if not parts:
        return
    with open(path, "a") as out:
        for name in parts:
            with open(os.path.join(d, name)) as fh:
                for line in fh:
                    if line.endswith("\n"):  # a torn last line was never complete
                        out.write(line)
    for name in parts:
        os.remove(os.path.join(d, name))


def gather_payloads(payload, device):
    """Every rank's packed bytes to rank 0: the byte counts with one all_gather
    (8 B per rank: every rank pads its buffer to the largest), then the padded
    buffers with one RCCL gather to rank 0.  Rank 0 returns every rank's bytes
    in rank order, the other ranks []."""
    import torch
    import torch.distributed as dist
    n = torch.tensor([len(payload)], dtype=torch.int64, device=device)
    sizes = [torch.zeros_like(n) for _ in range(dist.get_world_size())]
    dist.all_gather(sizes, n)
    cap = int(max(s.item() for s in sizes))
    buf = torch.zeros(max(cap, 1), dtype=torch.uint8, device=device)
    if payload:
        buf[:len(payload)] = torch.frombuffer(bytearray(payload), dtype=torch.uint8).to(device)
    root = dist.get_rank() == 0
    bufs = [torch.zeros_like(buf) for _ in sizes] if root else None
    dist.gather(buf, bufs, dst=0)
    if not root:
        return []
    return [b[:int(s.item())].cpu().numpy().tobytes() for s, b in zip(sizes, bufs)]


def gather_lines(lines, device):
    """Every rank's record lines to rank 0 (gather_payloads); rank 0 returns all
    lines, the other ranks []."""
    out = []
    for p in gather_payloads("\n".join(lines).encode(), device):
        if p:
            out.extend(p.decode().split("\n"))
    return out


def sort_payloads(payloads):
    """The lines of every payload (b"\\n"-separated record lines, as
    gather_payloads returns them) sorted like sort -k1,1 -k2,2n in the C locale
    (byte order, whole-line last resort; sort_lines' order for ASCII lines),
    joined by b"\\n".  Works on line offsets into the payloads: only the first
    two fields of a line are copied, so rank 0 of an N-GPU run sorts N x 100 MB
    of config-3 records without building a Python string per record."""
    offs, keys = [], []
    for k, p in enumerate(payloads):
        if not p:
            continue
        a, end = 0, len(p)
        while a <= end:
            b = p.find(b"\n", a)
            if b < 0:
                b = end
            t1 = p.find(b"\t", a, b)
            if t1 < 0:
                f0, v = p[a:b], b""
            else:
                t2 = p.find(b"\t", t1 + 1, b)
                f0, v = p[a:t1], p[t1 + 1:(t2 if t2 >= 0 else b)]
            if v.isdigit():
                num = int(v)
            else:
                m = re.match(rb"\s*([+-]?\d+)", v)
                num = int(m.group(1)) if m else 0
            keys.append((f0, num))
            offs.append((k, a, b))
            a = b + 1
    order = sorted(range(len(keys)), key=keys.__getitem__)
    # equal (field 1, field 2): whole lines decide, as sort's last resort
    i = 0
    while i < len(order):
        j = i + 1
        while j < len(order) and keys[order[j]] == keys[order[i]]:
            j += 1
        if j - i > 1:
            order[i:j] = sorted(order[i:j], key=lambda x: payloads[offs[x][0]][offs[x][1]:offs[x][2]])
        i = j
    views = [memoryview(p) for p in payloads]
    return b"\n".join(views[k][a:b] for k, a, b in (offs[x] for x in order))


def localGraph_npz(args):
    t0 = time.time()
    tsid = args.TSampleID.split(",")
    nsid = args.NSampleID.split(",")
    rawoutput = "%s.vs.%s.TandemRepeat.Raw.bed" % ("-".join(tsid), "-".join(nsid))
    path = os.path.join(args.savedir, rawoutput)
    cont = getattr(args, "Continue", False)
    world, rank, dist, device = _dist_setup()
    if rank == 0 and cont and os.path.exists(path):
        merge_parts(path)
    if dist is not None:
        dist.barrier()
    rows = load_bundles(args.savedir)
    finished = set()
    if cont and os.path.exists(path):
        with open(path) as fh:
            finished = {"\t".join(x.strip().split("\t")[0:3]) for x in fh if x.strip()}
    rows = [r for r in rows if window_key(r) not in finished]
    # a window past an engine limit fails alone: every other record is still
    # written, gathered and sorted on every rank, then the failures are raised
    failed = {}
    if dist is not None:
        # each rank journals its records as batches complete; rank 0 receives
        # every rank's records with one RCCL gather and writes the output
        owner = shard_lpt(rows, world)
        mine = [r for r, o in zip(rows, owner) if o == rank]
        lines = write_journal(part_path(path, rank), "w", mine, args.batch, failed)
    else:
        lines = write_journal(path, "a" if finished else "w", rows, args.batch, failed)
    out = _finish(path, lines, rank, world, dist, device, finished, t0, "Local Graph")
    _report_failed(failed, rank)
    return out


def _dist_setup():
    """(world, rank, dist or None, device): one process per GPU, RCCL between
    GPUs; gloo only for CPU rehearsals of the plumbing."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world <= 1:
        return world, rank, None, None
    # this rank's CPU slice and pool size, before its context exists
    from svscope_amd import hostcpu
    hostcpu.apply()
    import torch
    import torch.distributed as dist
    local = int(os.environ.get("LOCAL_RANK", "0"))
    gpu = torch.cuda.is_available()
    backend = os.environ.get("SVS_DIST_BACKEND") or ("nccl" if gpu else "gloo")
    device = torch.device("cpu")
    if gpu:
        ordinal = rank_device(backend, local, os.environ)
        torch.cuda.set_device(ordinal)
        os.environ["SVS_DEVICE"] = str(ordinal)
        if backend == "nccl":
            device = torch.device("cuda", ordinal)
    if not dist.is_initialized():
        dist.init_process_group(backend)
    return world, rank, dist, device


def rank_device(backend, local, env):
    """The GPU of this rank's engine (and, under nccl, its communicator):
    LOCAL_RANK.  Only with SVS_DIST_BACKEND=gloo (tests on a one-GPU box) does
    SVS_DEVICE=d put every rank's engine on GPU d, the records gathered over
    gloo on the host.  Under nccl a stale exported SVS_DEVICE would put every
    rank on one GPU, which RCCL rejects: it is ignored there, with
    a warning when it names another GPU."""
    dev = env.get("SVS_DEVICE")
    if backend == "gloo" and dev is not None:
        return int(dev)
    if dev is not None and int(dev) != local:
        log.warning("SVS_DEVICE=%s ignored under %s: rank with LOCAL_RANK %d uses GPU %d", dev, backend, local, local)
    return local


def _finish(path, lines_by_rank, rank, world, dist, device, finished, t0, what):
    """Multi-rank: gather every rank's journalled lines to rank 0 (an 8-B
    all_gather of the sizes, then one RCCL gather to rank 0), then rank 0
    sorts the output like sort -k1,1 -k2,2n."""
    if dist is not None:
        lines = gather_lines(lines_by_rank, device)
        if rank == 0:
            with open(path, "a" if finished else "w") as fh:
                fh.write("".join(line + "\n" for line in lines))
        dist.barrier()
        os.remove(part_path(path, rank))
    if rank == 0:
        with open(path) as fh:
            allines = [x.rstrip("\n") for x in fh if x.strip()]
        with open(path, "w") as fh:
            for line in sort_lines(allines):
                fh.write(line + "\n")
        log.info("%s : work finished with %s hour", what, (time.time() - t0) / 3600)
    return path


def localGraph(args, readers=None):
    """The BAM-reading localGraph (SVscope.py:118-183): window BED ->
    DataMaker -> Decision (+ the DUP corner re-scan, TDscope) -> Raw.bed.

    Extraction (data_maker.DataMaker / DataMaker2, BAM I/O) runs in a
    process pool of min(6, -p) spawned workers, as the reference caps its
    Pool (:158-161); each chunk of ``args.batch`` windows then goes through
    TDscope_batch (DecisionBatch on the GPU), the next chunk's extraction
    overlapping it.  Records are journalled per chunk (flushed), --Continue
    skips windows already written (the reference's check never matches,
    SURVEY.md §5), multi-GPU shards windows round-robin (their cost is unknown
    before extraction) with the same single RCCL gather as localGraph_npz.
    ``readers`` replaces pysam (data_maker's hook)."""
    import functools
    import multiprocessing as mp
    import sys
    from .data_maker import DataMaker, DataMaker2
    from .decision_maker import WindowFailed
    from .som_td_detector import TDscope_batch
    t0 = time.time()
    tumor, normal = args.Tumorbam.split(","), args.Normalbam.split(",")
    tsid, nsid = args.TSampleID.split(","), args.NSampleID.split(",")
    if len(tsid) != len(tumor):
        print("SampleID not meet tumor bam file, exit !")
        sys.exit(1)
    if len(nsid) != len(normal):
        print("SampleID not meet normal bam file, exit !")
        sys.exit(1)
    bams = tumor + normal
    labels = [x + "_tumor" for x in tsid] + [x + "_normal" for x in nsid]
    rawoutput = "%s.vs.%s.TandemRepeat.Raw.bed" % ("-".join(tsid), "-".join(nsid))
    if not os.path.exists(args.savedir):
        os.mkdir(args.savedir)
    path = os.path.join(args.savedir, rawoutput)
    with open(args.windowBed) as fh:
        records = ["\t".join(x.strip().split("\t")) for x in fh.readlines()]
    cont = getattr(args, "Continue", False)
    world, rank, dist, device = _dist_setup()
    if rank == 0 and cont and os.path.exists(path):
        merge_parts(path)
    if dist is not None:
        dist.barrier()
    finished = set()
    if cont and os.path.exists(path):
        with open(path) as fh:
            finished = {"\t".join(x.strip().split("\t")[0:3]) for x in fh if x.strip()}
    records = [r for r in records if "\t".join(r.split("\t")[0:3]) not in finished]
    mine = records[rank::world]
    dm = functools.partial(DataMaker, refFile=args.Reference, bamFileList=bams, LabelList=labels,
                           offset=int(args.offset), mapQ=int(args.mapQ), readers=readers)
    dm2 = functools.partial(DataMaker2, refFile=args.Reference, bamFileList=bams, LabelList=labels,
                            offset=int(args.offset), mapQ=int(args.mapQ), readers=readers)
    procs = min(6, int(args.thread))
    pool = mp.get_context("spawn").Pool(procs) if procs > 1 else None
    map_fn = pool.map if pool else map
    B = max(1, int(getattr(args, "batch", 512)))
    chunks = [mine[k:k + B] for k in range(0, len(mine), B)]
    out_path = part_path(path, rank) if dist is not None else path
    lines = []
    failed = {}  # windows past an engine limit: reported after the output is complete
    try:
        with open(out_path, "w" if dist is not None else ("a" if finished else "w")) as fh:
            nxt = pool.map_async(dm, chunks[0]) if (pool and chunks) else None
            for k, chunk in enumerate(chunks):
                bundles = nxt.get() if nxt is not None else [dm(r) for r in chunk]
                nxt = pool.map_async(dm, chunks[k + 1]) if (pool and k + 1 < len(chunks)) else None
                try:
                    recs = TDscope_batch(chunk, dm, dm2, map_fn=map_fn, bundles=bundles)
                except WindowFailed as e:
                    recs = e.records
                    failed.update({"\t".join(chunk[i].split("\t")[0:3]): why for i, why in e.failed.items()})
                chunk_lines = [record_line(x) for x in recs if x is not None]
                fh.write("".join(line + "\n" for line in chunk_lines))
                fh.flush()
                lines.extend(chunk_lines)
    finally:
        if pool:
            pool.close()
            pool.join()
    out = _finish(path, lines, rank, world, dist, device, finished, t0, "Local Graph")
    _report_failed(failed, rank)
    return out


def main(argv=None):
    """python -m svscope_amd.local_graph [localGraph|localGraph_npz] ...
    (the SVscope.py sub-commands of this path; localGraph_npz by default)."""
    import sys
    argv = list(sys.argv[1:] if argv is None else argv)
    cmd = argv.pop(0) if argv and argv[0] in ("localGraph", "localGraph_npz") else "localGraph_npz"
    ap = argparse.ArgumentParser(description="SVScope %s on MI355X" % cmd)
    if cmd == "localGraph":
        ap.add_argument("-w", "--windowBed", required=True)
        ap.add_argument("-T", "--Tumorbam", required=True)
        ap.add_argument("-N", "--Normalbam", required=True)
        ap.add_argument("-r", "--Reference", required=True)
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
    print(localGraph(args) if cmd == "localGraph" else localGraph_npz(args))


if __name__ == "__main__":
    main()
