"""Builds libsvscope_hip.so (HIP kernels for gfx950 + host engine + C ABI) in-tree.

    python -m svscope_amd.build          # -> svscope_amd/lib/libsvscope_hip.so

Sources are compiled with hipcc --offload-arch=gfx950 into objects under
build/ (parallel), then linked into one shared library with no torch types in
its interface.
"""
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
OBJ = os.path.join(ROOT, "build", "svscope_obj")
LIB_DIR = os.path.join(PKG, "lib")
LIB = os.path.join(LIB_DIR, "libsvscope_hip.so")
ARCH = os.environ.get("SVS_OFFLOAD_ARCH", "gfx950")

SOURCES = [
    "poa_strip.hip",
    "poa_prep.hip",
    "poa_fold.hip",
    "em_kernels.hip",
    "misscore_kernels.hip",
    "poa_graph.cpp",
    "svs_threadpool.cpp",
    "ward.cpp",
    "features.cpp",
    "svs_decision.cpp",
    "svs_poa_engine.cpp",
    "svs_em_engine.cpp",
    "svs_misscore_engine.cpp",
    "svs_abi.cpp",
]


def _hipcc():
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the MI355X engine cannot be built")


def _compile(src):
    path = os.path.join(CSRC, src)
    obj = os.path.join(OBJ, src.rsplit(".", 1)[0] + ".o")
    deps = [path] + [os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith(".hpp")]
    deps.append(os.path.join(ROOT, "include", "svscope.h"))
    if os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(d) for d in deps):
        return obj
    cmd = [_hipcc(), "-x", "hip", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
           "-Wall", "-Wno-unused-result", "-c", path, "-o", obj]
    if not src.endswith(".hip"):
        # host-only translation units: no device code, no device pass at all
        cmd = [_hipcc(), "-O3", "-std=c++17", "-fPIC", "-Wall", "-D__HIP_PLATFORM_AMD__",
               "--offload-host-only", "-c", path, "-o", obj]
    subprocess.check_call(cmd)
    return obj


def build(verbose=False):
    os.makedirs(OBJ, exist_ok=True)
    os.makedirs(LIB_DIR, exist_ok=True)
    srcs = [s for s in SOURCES if os.path.exists(os.path.join(CSRC, s))]
    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(_compile, srcs))
    if os.path.exists(LIB) and os.path.getmtime(LIB) >= max(os.path.getmtime(o) for o in objs):
        return LIB
    tmp = LIB + ".tmp"
    subprocess.check_call([_hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", tmp] + objs +
                          ["-lpthread"])
    os.replace(tmp, LIB)
    if verbose:
        print("built", LIB)
    return LIB


if __name__ == "__main__":
    build(verbose=True)
    sys.exit(0)
