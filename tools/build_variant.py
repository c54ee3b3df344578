"""Builds a development variant of libsvscope_hip.so with extra compile flags.

    python tools/build_variant.py NAME -DFLAG[=V] ...
    -> svscope_amd/lib/variants/libsvscope_hip_NAME.so  (select with SVS_LIB_PATH)

Objects go to build/variant_NAME/; the product library is not touched.
"""
import concurrent.futures as cf
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from svscope_amd import build as B  # noqa: E402


def main():
    name, flags = sys.argv[1], sys.argv[2:]
    obj_dir = os.path.join(ROOT, "build", "variant_" + name)
    os.makedirs(obj_dir, exist_ok=True)
    out_dir = os.path.join(B.LIB_DIR, "variants")
    os.makedirs(out_dir, exist_ok=True)

    def comp(src):
        obj = os.path.join(obj_dir, src.rsplit(".", 1)[0] + ".o")
        path = os.path.join(B.CSRC, src)
        if src.endswith(".hip"):
            cmd = [B._hipcc(), "-x", "hip", f"--offload-arch={B.ARCH}", "-O3", "-std=c++17", "-fPIC"]
        else:
            cmd = [B._hipcc(), "-O3", "-std=c++17", "-fPIC", "-D__HIP_PLATFORM_AMD__"]
        subprocess.check_call(cmd + flags + ["-c", path, "-o", obj])
        return obj

    with cf.ThreadPoolExecutor(max_workers=8) as ex:
        objs = list(ex.map(comp, B.SOURCES))
    lib = os.path.join(out_dir, f"libsvscope_hip_{name}.so")
    subprocess.check_call([B._hipcc(), "-shared", "-fPIC", f"--offload-arch={B.ARCH}", "-o", lib] + objs + ["-lpthread"])
    print(lib)


if __name__ == "__main__":
    main()
