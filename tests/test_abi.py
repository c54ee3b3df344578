"""C-ABI library: loads here (no GPU) and exports every symbol include/svscope.h declares."""
import ctypes
import os
import re

import pytest

from svscope_amd import _abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "svscope.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(svs_[a-z_0-9]+)\s*\(", src)))


def test_header_declares_entry_points():
    names = declared_functions()
    assert "svs_poa_batch" in names and "svs_init" in names


def test_library_exports_every_declared_symbol():
    lib = _abi.load_library()
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_no_device_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(_abi.SvsError):
        _abi.Context(0)


def test_last_error_is_string():
    lib = _abi.load_library()
    assert isinstance(lib.svs_last_error(), bytes)


def test_ctypes_structs_match_the_header_layout(tmp_path):
    """Every ctypes mirror of a public struct has the header's field offsets
    and size (a field removed from the middle of svs_poa_stats
    moved the ones after it), and the library reports the header's
    SVS_ABI_VERSION, which load_library checks."""
    import subprocess
    structs = {"svs_poa_stats": _abi.PoaStats, "svs_poa_config": _abi.PoaConfig, "svs_em_window": _abi.EmWindow,
               "svs_em_config": _abi.EmConfig, "svs_decision_window": _abi.DecisionWindow,
               "svs_decision_config": _abi.DecisionConfig, "svs_decision_stats": _abi.DecisionStats,
               "svs_misscore_stats": _abi.MisscoreStats}
    lines = ['#include <stddef.h>', '#include <stdio.h>', '#include "svscope.h"', "int main(void) {"]
    for cname, cls in structs.items():
        lines.append(f'  printf("{cname} size %zu\\n", sizeof({cname}));')
        for fname, _ in cls._fields_:
            lines.append(f'  printf("{cname} {fname} %zu\\n", offsetof({cname}, {fname}));')
    lines.append('  printf("version %d\\n", SVS_ABI_VERSION);')
    lines.append("  return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)])
    got = {}
    for line in subprocess.check_output([str(exe)]).decode().splitlines():
        *key, val = line.split()
        got[tuple(key)] = int(val)
    for cname, cls in structs.items():
        assert got[(cname, "size")] == ctypes.sizeof(cls), cname
        for fname, _ in cls._fields_:
            assert got[(cname, fname)] == getattr(cls, fname).offset, (cname, fname)
    assert got[("version",)] == _abi.ABI_VERSION == _abi.load_library().svs_abi_version()
