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
