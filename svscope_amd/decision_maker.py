"""Per-window somatic/germline decision, batched for the GPU.

``Decision(TDRecord, sequenceList, ReadIDs, flank_5, flank_3, windowFlag='NormalOutput',
Tlabel='tumor', readcutoff=3, hcutoff=3, scutoff=0.05) -> list[10]`` keeps the
signature, gate, labelling and record format of
/root/reference/src/DecisionMaker.py:110-191:
  gate :134 -> MSAFeatureSelection :136 -> EMCluster if >= 10 features :137-138
  -> per-cluster somatic/germline test in ascending label order :145-154
  -> POA consensus per reported cluster :155-176 -> record :178-190.
``DecisionBatch(windows, ...)`` runs the same logic for many windows through
one ``svs_decision_batch`` call: window MSAs, feature selection, EM and the
cluster consensus POAs are pipelined inside the engine (include/svscope.h).
"""
import ctypes
import os
import time

import numpy as np

from . import _abi


def _tag(read_id):
    return read_id.split("|")[0].split("_")[-1]


def _pack_windows(windows, gated, Tlabel):
    """Flattens the gated windows into the svs_decision_batch input arrays."""
    wins = (_abi.DecisionWindow * max(1, len(gated)))()
    byte_start = [0]
    chunks, text, tags = [], [], []
    total = text_len = tag_len = 0
    for k, w in enumerate(gated):
        rec, seqs, ids, f5, f3 = windows[w][:5]
        W = wins[k]
        W.n_seqs = len(seqs)
        W.n_ids = len(ids)
        W.seq_start = len(byte_start) - 1
        for s in seqs:
            b = s.encode("latin-1") if isinstance(s, str) else bytes(s)
            chunks.append(b)
            total += len(b)
            byte_start.append(total)
        b5, b3 = f5.encode("latin-1"), f3.encode("latin-1")
        W.flank5_off, W.flank5_len = text_len, len(b5)
        W.flank3_off, W.flank3_len = text_len + len(b5), len(b3)
        text.append(b5 + b3)
        text_len += len(b5) + len(b3)
        W.tag_off = tag_len
        tags.append(np.fromiter((_tag(x) == Tlabel for x in ids), dtype=np.uint8, count=len(ids)))
        tag_len += len(ids)
    starts = np.asarray(byte_start, dtype=np.int64)
    blob = b"".join(chunks) or b"\0"
    txt = b"".join(text) or b"\0"
    tag_arr = np.concatenate(tags) if tag_len else np.zeros(1, np.uint8)
    return wins, starts, blob, txt, tag_arr


def _config(readcutoff, hcutoff, scutoff):
    cfg = _abi.DecisionConfig()
    cfg.readcutoff, cfg.hcutoff, cfg.scutoff = int(readcutoff), int(hcutoff), float(scutoff)
    cfg.poa = _abi.PoaConfig(1, 5, -4, -8, -6, -10, -4, -1, 1)
    cfg.em = _abi.EmConfig(9, 20, 2023, 0, 1e-10)
    cfg.em_batch = int(os.environ.get("SVS_EM_BATCH", "0"))
    return cfg


def _gate(windows):
    """Default records and the indices of the windows that pass the gate (:127-134)."""
    records = []
    gated = []
    for w, win in enumerate(windows):
        rec, seqs, ids, f5, f3 = win[:5]
        flag = win[5] if len(win) > 5 else "NormalOutput"
        chrom, start, end = rec.strip().split("\t")[0:3]
        records.append([chrom, start, end, "-", "-", 0, "-", "-", 0, flag])
        if len(ids):
            tags, counts = np.unique(np.array([_tag(x) for x in ids]), return_counts=True)
        else:
            tags, counts = np.array([]), np.array([])
        if len(seqs) > 3 and tags.shape[0] >= 2 and np.min(counts) >= 3:
            gated.append(w)
    return records, gated


class WindowFailed(_abi.SvsError):
    """Some windows of a batch went past an engine limit (status
    SVS_DEC_FAILED): ``failed`` maps their batch indices to the reason,
    ``records`` holds every other window's finished record (None for the failed
    ones).  The reference has no such limits; the engine fails those windows
    alone and the caller decides what to write."""

    def __init__(self, failed, records):
        self.failed = dict(failed)
        self.records = records
        first = next(iter(self.failed.items()))
        super().__init__(f"{len(self.failed)} window(s) past an engine limit, window {first[0]}: {first[1]}")


def _format(lib, res, windows, gated, records):
    """Fills the records of the gated windows from a decision result (:178-190).
    Raises WindowFailed, after filling every other record, when windows went
    past an engine limit."""
    status, K, ns, ng = (ctypes.c_int32() for _ in range(4))
    failed = {}
    iptr = ctypes.POINTER(ctypes.c_int32)()
    nid = ctypes.c_int32()
    cptr = ctypes.c_void_p()
    clen = ctypes.c_int64()
    for k, w in enumerate(gated):
        _abi.check(lib.svs_decision_result_window(res, k, ctypes.byref(status), ctypes.byref(K),
                                                  ctypes.byref(ns), ctypes.byref(ng)))
        if status.value == _abi.DEC_INDEX_ERROR:
            raise IndexError(f"window {w}: an EM label row has no read id (the reference raises here)")
        if status.value == _abi.DEC_FAILED:
            msg = ctypes.c_char_p()
            _abi.check(lib.svs_decision_result_window_error(res, k, ctypes.byref(msg)))
            failed[w] = (msg.value or b"").decode()
            records[w] = None
            continue
        if status.value != _abi.DEC_EMOUTPUT:
            continue
        ids = windows[w][2]
        seqs_out, ids_out = [], []
        for c in range(ns.value + ng.value):
            _abi.check(lib.svs_decision_result_cluster(res, k, c, ctypes.byref(iptr), ctypes.byref(nid),
                                                       ctypes.byref(cptr), ctypes.byref(clen)))
            seqs_out.append(ctypes.string_at(cptr, clen.value).decode("ascii"))
            ids_out.append(",".join(str(ids[iptr[i]]) for i in range(nid.value)))
        r = records[w]
        r[3] = ";".join(seqs_out[:ns.value])
        r[4] = ";".join(ids_out[:ns.value])
        r[5] = ns.value
        r[6] = ";".join(seqs_out[ns.value:])
        r[7] = ";".join(ids_out[ns.value:])
        r[8] = ng.value
        r[9] = r[9] + "|EMOutput"
    if failed:
        raise WindowFailed(failed, records)
    return records


def _stats_entries(d, extra):
    phases = {"features_s": d["features_ms"] / 1e3, "labelling_s": d["labelling_ms"] / 1e3,
              "em_wall_s": d["em_wall_ms"] / 1e3, "em_kernel_s": d["em_kernel_ms"] / 1e3,
              "em_launches": d["em_launches"], "em_windows": d["em_windows"],
              "consensus_tasks": d["consensus_tasks"]}
    phases.update(extra)
    return [("decision_poa", d["poa"]), ("phases", phases)]


class DecisionSession:
    """Streaming DecisionBatch over one svs_decision_session (include/svscope.h).

    ``submit(windows)`` gates and packs a batch, queues it and returns a ticket
    at once; ``wait(ticket)`` returns its records.  The engine keeps one POA
    scheduler for every submitted batch, so batch b+1's window MSAs fill the GPU
    while batch b's EM and consensus finish.  This replaces the reference's
    ``Pool.imap_unordered(TDscope_npz, ...)`` fan-out (SVscope.py:220-233).
    """

    def __init__(self, context=None, Tlabel="tumor", readcutoff=3, hcutoff=3, scutoff=0.05):
        self.ctx = context or _abi.default_context()
        self.lib = self.ctx.lib
        self.Tlabel = Tlabel
        self.cfg = _config(readcutoff, hcutoff, scutoff)
        h = ctypes.c_void_p()
        _abi.check(self.lib.svs_decision_session_open(self.ctx.handle, ctypes.byref(self.cfg), ctypes.byref(h)),
                   "svs_decision_session_open")
        self.handle = h
        self._pending = {}
        self._local = 0  # tickets of batches with no gated window (never reach the engine)

    def submit(self, windows):
        windows = list(windows)
        records, gated = _gate(windows)
        if not gated:
            self._local -= 1
            self._pending[self._local] = (windows, gated, records, None)
            return self._local
        packed = _pack_windows(windows, gated, self.Tlabel)
        wins, starts, blob, txt, tag_arr = packed
        ticket = ctypes.c_int64()
        _abi.check(self.lib.svs_decision_session_submit(
            self.handle, len(gated), wins, starts.ctypes.data_as(ctypes.c_void_p), blob, txt,
            tag_arr.ctypes.data_as(ctypes.c_void_p), ctypes.byref(ticket)), "svs_decision_session_submit")
        # the engine reads the packed arrays until the batch is waited for
        self._pending[ticket.value] = (windows, gated, records, packed)
        return ticket.value

    def wait(self, ticket):
        windows, gated, records, packed = self._pending.pop(ticket)
        if packed is None:
            return records
        res = ctypes.c_void_p()
        _abi.check(self.lib.svs_decision_session_wait(self.handle, ctypes.c_int64(ticket), ctypes.byref(res)),
                   "svs_decision_session_wait")
        try:
            return _format(self.lib, res, windows, gated, records)
        finally:
            self.lib.svs_decision_result_free(res)

    def stats(self):
        st = _abi.DecisionStats()
        _abi.check(self.lib.svs_decision_session_stats(self.handle, ctypes.byref(st)), "svs_decision_session_stats")
        return st.as_dict()

    def close(self):
        if getattr(self, "handle", None):
            h, self.handle = self.handle, None
            _abi.check(self.lib.svs_decision_session_close(h), "svs_decision_session_close")
            self._pending.clear()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def DecisionBatch(windows, Tlabel="tumor", readcutoff=3, hcutoff=3, scutoff=0.05, context=None, stats=None):
    """windows: list of (TDRecord, sequenceList, ReadIDs, flank_5, flank_3[, windowFlag]).
    Returns the list of 10-field records, in input order.  The gated windows go
    through one svs_decision_batch call (MSA POA, features, EM and consensus
    POA pipelined on the GPU); this function keeps the gate (:134) and the
    record formatting (:178-190)."""
    t_start = time.perf_counter()
    records, gated = _gate(windows)
    if not gated:
        return records
    ctx = context or _abi.default_context()
    lib = ctx.lib
    wins, starts, blob, txt, tag_arr = _pack_windows(windows, gated, Tlabel)
    cfg = _config(readcutoff, hcutoff, scutoff)
    res = ctypes.c_void_p()
    t0 = time.perf_counter()
    _abi.check(lib.svs_decision_batch(ctx.handle, len(gated), wins, starts.ctypes.data_as(ctypes.c_void_p), blob, txt,
                                      tag_arr.ctypes.data_as(ctypes.c_void_p), ctypes.byref(cfg), ctypes.byref(res)),
               "svs_decision_batch")
    t1 = time.perf_counter()
    try:
        _format(lib, res, windows, gated, records)
        if stats is not None:
            st = _abi.DecisionStats()
            _abi.check(lib.svs_decision_result_stats(res, ctypes.byref(st)))
            stats.extend(_stats_entries(st.as_dict(), {"decision_call_s": t1 - t0,
                                                       "format_s": time.perf_counter() - t1,
                                                       "decision_total_s": time.perf_counter() - t_start}))
    finally:
        lib.svs_decision_result_free(res)
    return records


def Decision(TDRecord, sequenceList, ReadIDs, flank_5, flank_3, windowFlag="NormalOutput", Tlabel="tumor",
             readcutoff=3, hcutoff=3, scutoff=0.05):
    return DecisionBatch([(TDRecord, sequenceList, ReadIDs, flank_5, flank_3, windowFlag)], Tlabel, readcutoff,
                         hcutoff, scutoff)[0]
