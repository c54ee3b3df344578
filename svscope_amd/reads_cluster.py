"""Drop-in for the reference's ReadsCluster.EMCluster, executed on MI355X.

``EMCluster(seqdatamx, initselection=1, max_C=9, ShowPlot=False)
-> [K, seqdatamx, Rclust, thetap, gamma, pie, BICList]``
(/root/reference/src/ReadsCluster.py:221-277, called at DecisionMaker.py:138).

Pipeline per batch of windows:
  1. read similarity S (pariwiseDistance, :52-59)           -> HIP kernel
  2. scipy ward linkage(S) + fcluster(K, 'maxclust') (:243, :94) -> host C++
     restatement on the engine thread pool (csrc/ward.cpp; bit-exact vs scipy,
     tests/test_ward_host.py)
  3. EM for K = 1..Kmax-1, BIC, K=1->2 rule, argmax (:246-277) -> HIP kernel
Only ``initselection=1`` (the value the reference uses) is implemented.
RNG contract: each window starts from numpy's RandomState(2023) stream
(SURVEY.md §8(a15)); the per-window stream offset consumed is reported.
"""
import ctypes
import time

import numpy as np

from . import _abi


EmWindowStruct = _abi.EmWindow
EmConfigStruct = _abi.EmConfig


_F_K, _F_RCLUST, _F_BIC, _F_LIK, _F_GAMMA, _F_PI, _F_THETA, _F_RNG = range(8)


def _pack_matrices(mats):
    wins = (EmWindowStruct * max(1, len(mats)))()
    offs = 0
    blobs = []
    for w, X in enumerate(mats):
        n, nf = X.shape
        wins[w].n_reads = n
        wins[w].n_feat = nf
        wins[w].x_off = offs
        blobs.append(np.ascontiguousarray(X, dtype=np.uint8).reshape(-1))
        offs += n * nf
    blob = np.concatenate(blobs) if blobs else np.zeros(1, np.uint8)
    if blob.size == 0:
        blob = np.zeros(1, np.uint8)
    return wins, blob


def similarity_batch(mats, context=None):
    """GPU pariwiseDistance for each N x nf matrix; returns list of N x N float64."""
    ctx = context or _abi.default_context()
    if not mats:
        return []
    wins, blob = _pack_matrices(mats)
    s_off = np.zeros(len(mats), np.int64)
    tot = 0
    for w, X in enumerate(mats):
        s_off[w] = tot
        tot += X.shape[0] ** 2
    S = np.zeros(max(1, tot), np.float64)
    _abi.check(ctx.lib.svs_similarity_batch(ctx.handle, len(mats), wins,
                                            blob.ctypes.data_as(ctypes.c_void_p),
                                            s_off.ctypes.data_as(ctypes.c_void_p),
                                            S.ctypes.data_as(ctypes.c_void_p)), "svs_similarity_batch")
    return [S[s_off[w]:s_off[w] + X.shape[0] ** 2].reshape(X.shape[0], X.shape[0]) for w, X in enumerate(mats)]


def em_cluster_batch(mats, max_C=9, n_step=20, seed=2023, want_params=False, context=None, timing=None):
    """Batched EMCluster.  Returns one dict per matrix:
    K, Rclust, BICList, lik (+ gamma, pi, theta when want_params)."""
    ctx = context or _abi.default_context()
    mats = [np.asarray(X) for X in mats]
    for X in mats:
        if X.ndim != 2 or X.shape[0] < 3:
            raise ValueError("EMCluster needs an N x nf matrix with N >= 3 (BICList[1] is read at :270)")
        if X.size and (X.min() < 0 or X.max() > 4):
            raise ValueError("seqdatamx symbols must be 0..4 (DataScanner.SeqEncoder)")
    if not mats:
        return []
    t0 = time.perf_counter()
    wins, blob = _pack_matrices(mats)
    cfg = EmConfigStruct(int(max_C), int(n_step), int(seed), 1 if want_params else 0, 1e-10)
    res = ctypes.c_void_p()
    _abi.check(ctx.lib.svs_em_cluster_batch(ctx.handle, len(mats), wins, blob.ctypes.data_as(ctypes.c_void_p),
                                            ctypes.byref(cfg), ctypes.byref(res)), "svs_em_cluster_batch")
    if timing is not None:
        timing["em_cluster_call_s"] = time.perf_counter() - t0
    out = []
    try:
        if timing is not None:
            kms, reruns = ctypes.c_double(), ctypes.c_int64()
            _abi.check(ctx.lib.svs_em_result_stats(res, ctypes.byref(kms), ctypes.byref(reruns)))
            timing["em_kernel_ms"] = kms.value
            timing["em_reruns"] = reruns.value
        ptr = ctypes.c_void_p()
        cnt = ctypes.c_int64()

        def get(w, field, ctype, np_dtype):
            _abi.check(ctx.lib.svs_em_result_get(res, w, field, ctypes.byref(ptr), ctypes.byref(cnt)))
            n = cnt.value
            if n == 0:
                return np.zeros(0, np_dtype)
            arr = ctypes.cast(ptr, ctypes.POINTER(ctype * n)).contents
            return np.frombuffer(arr, dtype=np_dtype, count=n).copy()

        for w, X in enumerate(mats):
            N, nf = X.shape
            d = dict(K=int(get(w, _F_K, ctypes.c_int32, np.int32)[0]),
                     Rclust=get(w, _F_RCLUST, ctypes.c_int32, np.int32).astype(np.int64),
                     BICList=get(w, _F_BIC, ctypes.c_double, np.float64),
                     lik=get(w, _F_LIK, ctypes.c_double, np.float64),
                     rng_used=int(get(w, _F_RNG, ctypes.c_int64, np.int64)[0]))
            if want_params:
                K = d["K"]
                d["gamma"] = get(w, _F_GAMMA, ctypes.c_double, np.float64).reshape(N, K)
                d["pi"] = get(w, _F_PI, ctypes.c_double, np.float64)
                d["theta"] = get(w, _F_THETA, ctypes.c_double, np.float64).reshape(K, nf, 5)
            out.append(d)
    finally:
        ctx.lib.svs_em_result_free(res)
    return out


def EMCluster(seqdatamx, initselection=1, max_C=9, ShowPlot=False):
    """ReadsCluster.EMCluster signature and return list (:221-277)."""
    if initselection != 1:
        raise NotImplementedError("only initselection=1 (hierarchical init, as the reference calls it) is implemented")
    r = em_cluster_batch([seqdatamx], max_C=max_C, want_params=True)[0]
    return [r["K"], seqdatamx, r["Rclust"], r["theta"], r["gamma"], r["pi"], r["BICList"]]
