"""Times the batched GPU POA on synthetic windows (window MSA only)."""
import argparse
import json
import sys
import time
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from svscope_amd import synth
from svscope_amd.poa import poa_batch

ap = argparse.ArgumentParser()
ap.add_argument("--windows", type=int, default=64)
ap.add_argument("--reads", type=int, default=64)
ap.add_argument("--ref-len", type=int, default=3000)
ap.add_argument("--check", type=int, default=0, help="oracle-check this many windows")
a = ap.parse_args()
t = time.time()
wins = [synth.make_window(w, a.reads, a.ref_len) for w in range(a.windows)]
print(f"synth {time.time() - t:.1f}s", flush=True)
poa_batch([wins[0][0][:3]])  # warm up context
t = time.time()
out, st = poa_batch([w[0] for w in wins], return_stats=True)
wall = time.time() - t
st["windows_per_s"] = a.windows / wall
st["gcups_kernel"] = st["dp_cells"] / (st["kernel_ms"] * 1e-3) / 1e9
st["gcups_computed"] = st["cells_computed"] / (st["kernel_ms"] * 1e-3) / 1e9
st["computed_frac"] = st["cells_computed"] / max(1, st["dp_cells"])
st["wall_s"] = wall
if os.environ.get("SVS_STRIP_PROF"):
    import ctypes
    from svscope_amd import _abi
    lib = _abi.load_library()
    buf = (ctypes.c_ulonglong * 10)()
    lib.svs_debug_strip_prof.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.svs_debug_strip_prof(buf, 0)
    # poa_strip.hip SVS_STRIP_PROF: shader clocks summed over waves (ff and
    # waits nest in sweeps; the traceback is wave 0's), strip rows computed
    names = ["fetch_wait_cyc", "ff_cyc", "sweep_cyc", "tb_cyc", "end_barrier_cyc", "life_cyc", "rows_computed", "waves",
             "ff_wait_cyc", "unused"]
    st["strip_prof"] = dict(zip(names, list(buf)))
print(json.dumps(st), flush=True)
if a.check:
    from oracle.spoa_oracle import poa as oracle_poa
    for w, g in zip(wins[:a.check], out):
        assert g == oracle_poa(w[0], 1), "MISMATCH"
    print("oracle check ok", a.check)
