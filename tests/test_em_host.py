"""Host-side pieces of the EM seam that need no GPU."""
import ctypes

import numpy as np

from svscope_amd import _abi


def test_rng_table_is_numpy_legacy_bitwise():
    lib = _abi.load_library()
    n = 100_000
    out = np.zeros(n, np.float64)
    _abi.check(lib.svs_rng_exponential_table(2023, n, out.ctypes.data_as(ctypes.c_void_p)))
    np.testing.assert_array_equal(out, np.random.RandomState(2023).standard_exponential(n))
    _abi.check(lib.svs_rng_exponential_table(7, 1000, out.ctypes.data_as(ctypes.c_void_p)))
    np.testing.assert_array_equal(out[:1000], np.random.RandomState(7).standard_exponential(1000))


def test_ward_labels_shape():
    from test_ward_host import engine_labels
    from oracle.em_oracle import similarity
    rs = np.random.RandomState(0)
    X = rs.randint(0, 5, size=(12, 30))
    lab = engine_labels([similarity(X)])[0]
    assert lab.shape == (9, 12) and lab.min() >= 1 and (lab[0] == 1).all()
