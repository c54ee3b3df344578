"""ORACLE — test infrastructure only (see oracle/spoa_oracle.cpp header).

ctypes binding of the CPU spoa restatement with pyspoa 0.2.1's call signature
``poa(sequences, algorithm=0, genmsa=True, m=5, n=-4, g=-8, e=-6, q=-10, c=-4,
min_coverage=-1) -> (consensus, msa)`` as used by the reference at
/root/reference/src/DataScanner.py:206,213 and DecisionMaker.py:160,171.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  The product (svscope_amd) never does.
"""
import ctypes
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle_spoa.so")
_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def _load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(_LIB_PATH):
        build()
    lib = ctypes.CDLL(_LIB_PATH)
    lib.oracle_poa.restype = ctypes.c_void_p
    lib.oracle_poa.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_int)] + \
        [ctypes.c_int] * 8
    for name in ("oracle_error", "oracle_consensus"):
        getattr(lib, name).restype = ctypes.c_char_p
        getattr(lib, name).argtypes = [ctypes.c_void_p]
    lib.oracle_msa_row.restype = ctypes.c_char_p
    lib.oracle_msa_row.argtypes = [ctypes.c_void_p, ctypes.c_int]
    for name in ("oracle_consensus_len", "oracle_msa_rows", "oracle_msa_cols", "oracle_max_nodes"):
        getattr(lib, name).restype = ctypes.c_int
        getattr(lib, name).argtypes = [ctypes.c_void_p]
    lib.oracle_cells.restype = ctypes.c_ulonglong
    lib.oracle_cells.argtypes = [ctypes.c_void_p]
    lib.oracle_free.restype = None
    lib.oracle_free.argtypes = [ctypes.c_void_p]
    _lib = lib
    return lib


def poa_stats(sequences, algorithm=1, m=5, n=-4, g=-8, e=-6, q=-10, c=-4, min_coverage=-1):
    """Returns (consensus, msa, dp_cells, max_graph_nodes)."""
    lib = _load()
    enc = [s.encode("ascii") for s in sequences]
    arr = (ctypes.c_char_p * max(1, len(enc)))(*enc)
    lens = (ctypes.c_int * max(1, len(enc)))(*[len(s) for s in enc])
    h = lib.oracle_poa(len(enc), arr, lens, algorithm, m, n, g, e, q, c, min_coverage)
    try:
        err = lib.oracle_error(h)
        if err is not None:
            raise RuntimeError(err.decode())
        cons = lib.oracle_consensus(h).decode()
        msa = [lib.oracle_msa_row(h, i).decode() for i in range(lib.oracle_msa_rows(h))]
        return cons, msa, int(lib.oracle_cells(h)), int(lib.oracle_max_nodes(h))
    finally:
        lib.oracle_free(h)


def poa(sequences, algorithm=0, genmsa=True, m=5, n=-4, g=-8, e=-6, q=-10, c=-4, min_coverage=-1):
    cons, msa, _, _ = poa_stats(list(sequences), algorithm, m, n, g, e, q, c, min_coverage)
    return cons, (msa if genmsa else [])
