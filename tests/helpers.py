"""Shared test helpers (test infrastructure)."""
import ctypes
import os
import random
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EMU_SRC = [os.path.join(ROOT, "tests", "cpp", "kernel_emu.cpp"),
           os.path.join(ROOT, "svscope_amd", "csrc", "poa_graph.cpp")]
EMU_LIB = os.path.join(ROOT, "tests", "build", "libkernel_emu.so")


def random_poa_case(rnd, max_seqs=8, max_len=30, edits=6):
    k = rnd.randint(1, max_seqs)
    base = "".join(rnd.choice("ACGT") for _ in range(rnd.randint(0, max_len)))
    seqs = []
    for _ in range(k):
        s = list(base)
        for _ in range(rnd.randint(0, edits)):
            op = rnd.random()
            p = rnd.randint(0, max(0, len(s)))
            if op < 0.3 and s:
                s.pop(min(p, len(s) - 1))
            elif op < 0.6:
                s.insert(p, rnd.choice("ACGT"))
            elif s:
                s[min(p, len(s) - 1)] = rnd.choice("ACGT")
        if rnd.random() < 0.1:
            s = []
        if rnd.random() < 0.05:
            s = list(rnd.choice(["AAAAAAA", "ACACACAC", "T"]))
        seqs.append("".join(s))
    return seqs


def random_cases(seed, n, **kw):
    rnd = random.Random(seed)
    return [random_poa_case(rnd, **kw) for _ in range(n)]


def build_emu():
    os.makedirs(os.path.dirname(EMU_LIB), exist_ok=True)
    if not os.path.exists(EMU_LIB) or os.path.getmtime(EMU_LIB) < max(os.path.getmtime(s) for s in EMU_SRC):
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-o", EMU_LIB] + EMU_SRC)
    lib = ctypes.CDLL(EMU_LIB)
    lib.emu_poa.restype = ctypes.c_void_p
    lib.emu_poa.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_int)] + \
        [ctypes.c_int] * 6
    for n in ("emu_error", "emu_consensus"):
        getattr(lib, n).restype = ctypes.c_char_p
        getattr(lib, n).argtypes = [ctypes.c_void_p]
    lib.emu_msa_row.restype = ctypes.c_char_p
    lib.emu_msa_row.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.emu_msa_rows.argtypes = [ctypes.c_void_p]
    lib.emu_max_slots.argtypes = [ctypes.c_void_p]
    lib.emu_free.argtypes = [ctypes.c_void_p]
    return lib


def emu_poa(lib, seqs, m=5, n=-4, g=-8, e=-6, q=-10, c=-4):
    enc = [s.encode() for s in seqs]
    k = max(1, len(enc))
    h = lib.emu_poa(len(enc), (ctypes.c_char_p * k)(*enc), (ctypes.c_int * k)(*[len(s) for s in enc]),
                    m, n, g, e, q, c)
    try:
        err = lib.emu_error(h)
        if err:
            raise RuntimeError(err.decode())
        return lib.emu_consensus(h).decode(), [lib.emu_msa_row(h, i).decode() for i in range(lib.emu_msa_rows(h))]
    finally:
        lib.emu_free(h)
