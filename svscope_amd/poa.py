"""Drop-in for ``from spoa import poa`` (pyspoa 0.2.1), executed on MI355X.

``poa(sequences, algorithm=0, genmsa=True, m=5, n=-4, g=-8, e=-6, q=-10, c=-4,
min_coverage=-1) -> (consensus, msa)`` keeps pyspoa's signature and meaning;
the reference always calls it as ``poa(list, 1)``
(/root/reference/src/DataScanner.py:206,213, DecisionMaker.py:160,171).
Differences: only algorithm=1 (global NW) with spoa's convex gap subtype is
implemented (anything else raises), and there is no CPU path.

``poa_batch(list_of_sequence_lists, ...)`` runs many independent POA jobs in
one lockstep GPU pipeline (the batched seam used by DecisionBatch).
"""
import ctypes

from . import _abi


def _config(algorithm, genmsa, m, n, g, e, q, c, min_coverage):
    return _abi.PoaConfig(int(algorithm), int(m), int(n), int(g), int(e), int(q), int(c), int(min_coverage),
                          1 if genmsa else 0)


def _pack(jobs):
    job_start = [0]
    byte_start = [0]
    chunks = []
    total = 0
    for seqs in jobs:
        for s in seqs:
            b = s.encode("ascii") if isinstance(s, str) else bytes(s)
            chunks.append(b)
            total += len(b)
            byte_start.append(total)
        job_start.append(len(byte_start) - 1)
    blob = b"".join(chunks)
    js = (ctypes.c_int64 * len(job_start))(*job_start)
    bs = (ctypes.c_int64 * len(byte_start))(*byte_start)
    return js, bs, blob


def poa_batch(jobs, algorithm=1, genmsa=True, m=5, n=-4, g=-8, e=-6, q=-10, c=-4, min_coverage=-1,
              context=None, return_stats=False):
    """Runs len(jobs) independent POAs; returns [(consensus, msa), ...]."""
    ctx = context or _abi.default_context()
    lib = ctx.lib
    jobs = [list(j) for j in jobs]
    js, bs, blob = _pack(jobs)
    cfg = _config(algorithm, genmsa, m, n, g, e, q, c, min_coverage)
    res = ctypes.c_void_p()
    _abi.check(lib.svs_poa_batch(ctx.handle, len(jobs), js, bs, blob, ctypes.byref(cfg), ctypes.byref(res)),
               "svs_poa_batch")
    out = []
    try:
        ptr = ctypes.c_void_p()
        ln = ctypes.c_int64()
        rows = ctypes.c_int32()
        cols = ctypes.c_int32()
        for j in range(len(jobs)):
            _abi.check(lib.svs_poa_result_consensus(res, j, ctypes.byref(ptr), ctypes.byref(ln)))
            cons = ctypes.string_at(ptr, ln.value).decode("ascii") if ln.value else ""
            msa = []
            if genmsa:
                _abi.check(lib.svs_poa_result_msa(res, j, ctypes.byref(rows), ctypes.byref(cols), ctypes.byref(ptr)))
                if rows.value:
                    blk = ctypes.string_at(ptr, rows.value * cols.value).decode("ascii")
                    w = cols.value
                    msa = [blk[r * w:(r + 1) * w] for r in range(rows.value)]
            out.append((cons, msa))
        stats = _abi.PoaStats()
        _abi.check(lib.svs_poa_result_stats(res, ctypes.byref(stats)))
    finally:
        lib.svs_poa_result_free(res)
    if return_stats:
        return out, stats.as_dict()
    return out


def poa(sequences, algorithm=0, genmsa=True, m=5, n=-4, g=-8, e=-6, q=-10, c=-4, min_coverage=-1):
    """pyspoa-compatible single POA (see module docstring)."""
    return poa_batch([list(sequences)], algorithm, genmsa, m, n, g, e, q, c, min_coverage)[0]
