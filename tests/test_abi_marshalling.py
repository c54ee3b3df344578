"""Every ctypes prototype is exercised on CPU: a NULL context must come back
as SVS_E_INVALID (-1) before any device work, proving the argument lists
marshal (arity and types) exactly as include/svscope.h declares them."""
import ctypes

import numpy as np

from svscope_amd import _abi

NULL = ctypes.c_void_p()


def test_poa_batch_marshalling():
    lib = _abi.load_library()
    js = (ctypes.c_int64 * 2)(0, 1)
    bs = (ctypes.c_int64 * 2)(0, 4)
    cfg = _abi.PoaConfig(1, 5, -4, -8, -6, -10, -4, -1, 1)
    out = ctypes.c_void_p()
    assert lib.svs_poa_batch(NULL, 1, js, bs, b"ACGT", ctypes.byref(cfg), ctypes.byref(out)) == -1
    p = ctypes.c_void_p()
    n = ctypes.c_int64()
    r = ctypes.c_int32()
    assert lib.svs_poa_result_consensus(NULL, 0, ctypes.byref(p), ctypes.byref(n)) == -1
    assert lib.svs_poa_result_msa(NULL, 0, ctypes.byref(r), ctypes.byref(r), ctypes.byref(p)) == -1
    st = _abi.PoaStats()
    assert lib.svs_poa_result_stats(NULL, ctypes.byref(st)) == -1
    lib.svs_poa_result_free(NULL)


def test_em_marshalling():
    lib = _abi.load_library()
    wins = (_abi.EmWindow * 1)()
    wins[0].n_reads, wins[0].n_feat = 4, 3
    X = np.zeros(12, np.uint8)
    lab = np.ones(12, np.int32)
    s_off = np.zeros(1, np.int64)
    S = np.zeros(16)
    vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    assert lib.svs_similarity_batch(NULL, 1, wins, vp(X), vp(s_off), vp(S)) == -1
    cfg = _abi.EmConfig(9, 20, 2023, 0, 1e-10)
    out = ctypes.c_void_p()
    assert lib.svs_em_batch(NULL, 1, wins, vp(X), vp(lab), ctypes.byref(cfg), ctypes.byref(out)) == -1
    p = ctypes.c_void_p()
    n = ctypes.c_int64()
    assert lib.svs_em_result_get(NULL, 0, 0, ctypes.byref(p), ctypes.byref(n)) == -1
    lib.svs_em_result_free(NULL)


def test_context_marshalling():
    lib = _abi.load_library()
    x = np.zeros(64, np.int32)
    vp = x.ctypes.data_as(ctypes.c_void_p)
    assert lib.svs_wave_selftest(NULL, vp, vp, vp, 1) == -1
    n = ctypes.c_int()
    lib.svs_device_count(ctypes.byref(n))  # 0 devices on CPU, any count on GPU
    lib.svs_release(NULL)
