"""ctypes binding of libsvscope_hip.so (C ABI declared in include/svscope.h).

The library is built in-tree by svscope_amd.build.  There is no CPU fallback:
if the library or a HIP device is missing, every entry point raises.
"""
import ctypes
import os
import threading

LIB_PATH = os.environ.get("SVS_LIB_PATH") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libsvscope_hip.so")  # SVS_LIB_PATH: development variants

SVS_OK = 0
_ERRNAMES = {-1: "SVS_E_INVALID", -2: "SVS_E_NOMEM", -3: "SVS_E_HIP", -4: "SVS_E_UNSUPPORTED",
             -5: "SVS_E_INTERNAL"}



class SvsError(RuntimeError):
    pass


class PoaConfig(ctypes.Structure):
    _fields_ = [("algorithm", ctypes.c_int32), ("m", ctypes.c_int32), ("n", ctypes.c_int32),
                ("g", ctypes.c_int32), ("e", ctypes.c_int32), ("q", ctypes.c_int32), ("c", ctypes.c_int32),
                ("min_coverage", ctypes.c_int32), ("genmsa", ctypes.c_int32)]


class EmWindow(ctypes.Structure):
    _fields_ = [("n_reads", ctypes.c_int32), ("n_feat", ctypes.c_int32), ("x_off", ctypes.c_int64),
                ("label_off", ctypes.c_int64)]


class EmConfig(ctypes.Structure):
    _fields_ = [("max_c", ctypes.c_int32), ("n_step", ctypes.c_int32), ("seed", ctypes.c_int32),
                ("want_params", ctypes.c_int32), ("eps", ctypes.c_double)]


class PoaStats(ctypes.Structure):
    _fields_ = [("dp_cells", ctypes.c_uint64), ("alignments", ctypes.c_uint64), ("launches", ctypes.c_uint64),
                ("tb_bytes", ctypes.c_uint64), ("pool_bytes", ctypes.c_uint64), ("h2d_bytes", ctypes.c_uint64),
                ("d2h_bytes", ctypes.c_uint64), ("kernel_ms", ctypes.c_double), ("host_graph_ms", ctypes.c_double),
                ("wall_ms", ctypes.c_double), ("gpu_wait_ms", ctypes.c_double),
                ("cells_computed", ctypes.c_uint64), ("prune_retries", ctypes.c_uint64),
                ("prep_ms", ctypes.c_double), ("prep_jobs", ctypes.c_uint64),
                ("fold_ms", ctypes.c_double), ("fold_jobs", ctypes.c_uint64), ("wide_launches", ctypes.c_uint64),
                ("fold_update_ms", ctypes.c_double), ("fold_sort_ms", ctypes.c_double),
                ("fold_final_ms", ctypes.c_double), ("fold_prep_ms", ctypes.c_double),
                ("deferred_tasks", ctypes.c_uint64),
                ("dgraph_peak_bytes", ctypes.c_uint64), ("dgraph_reserved_bytes", ctypes.c_uint64),
                ("kernel_busy_ms", ctypes.c_double), ("dp_to_done_ms", ctypes.c_double)]

    def as_dict(self):
        return {name: getattr(self, name) for name, _ in self._fields_}


class DecisionWindow(ctypes.Structure):
    _fields_ = [("n_seqs", ctypes.c_int32), ("n_ids", ctypes.c_int32), ("seq_start", ctypes.c_int64),
                ("flank5_off", ctypes.c_int64), ("flank3_off", ctypes.c_int64), ("flank5_len", ctypes.c_int32),
                ("flank3_len", ctypes.c_int32), ("tag_off", ctypes.c_int64)]


class DecisionConfig(ctypes.Structure):
    _fields_ = [("readcutoff", ctypes.c_int32), ("hcutoff", ctypes.c_int32), ("scutoff", ctypes.c_double),
                ("poa", PoaConfig), ("em", EmConfig), ("em_batch", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class DecisionStats(ctypes.Structure):
    _fields_ = [("poa", PoaStats), ("wall_ms", ctypes.c_double), ("features_ms", ctypes.c_double),
                ("labelling_ms", ctypes.c_double), ("em_wall_ms", ctypes.c_double), ("em_kernel_ms", ctypes.c_double),
                ("msa_tasks", ctypes.c_int64), ("consensus_tasks", ctypes.c_int64), ("em_windows", ctypes.c_int64),
                ("em_launches", ctypes.c_int64), ("em_flops", ctypes.c_double), ("em_reruns", ctypes.c_int64)]

    def as_dict(self):
        d = {name: getattr(self, name) for name, _ in self._fields_ if name != "poa"}
        d["poa"] = self.poa.as_dict()
        return d


DEC_NO_EM, DEC_EM, DEC_EMOUTPUT, DEC_INDEX_ERROR, DEC_FAILED = 0, 1, 2, 3, 4


class MisscoreStats(ctypes.Structure):
    _fields_ = [("pairs", ctypes.c_uint64), ("dp_cells", ctypes.c_uint64), ("nib_bytes", ctypes.c_uint64),
                ("launches", ctypes.c_uint64), ("tb_steps", ctypes.c_uint64), ("fill_ms", ctypes.c_double),
                ("traceback_ms", ctypes.c_double), ("wall_ms", ctypes.c_double)]

    def as_dict(self):
        return {name: getattr(self, name) for name, _ in self._fields_}


MS_OK, MS_EMPTY = 0, 4

_lib = None
_lib_lock = threading.Lock()


ABI_VERSION = 6  # SVS_ABI_VERSION of include/svscope.h


def load_library():
    """Loads libsvscope_hip.so and declares its prototypes (no device needed)."""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise SvsError(f"{LIB_PATH} is missing: build it with `python -m svscope_amd.build` "
                           "(the MI355X engine has no CPU fallback)")
        lib = ctypes.CDLL(LIB_PATH)
        P, I32, I64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
        # the struct layouts below are those of include/svscope.h at ABI_VERSION
        lib.svs_abi_version.argtypes = []
        lib.svs_abi_version.restype = ctypes.c_int
        if lib.svs_abi_version() != ABI_VERSION:
            raise SvsError(f"{LIB_PATH} has ABI version {lib.svs_abi_version()}, this binding expects "
                           f"{ABI_VERSION}: rebuild it with `python -m svscope_amd.build`")
        lib.svs_init.argtypes = [ctypes.c_int, ctypes.POINTER(P)]
        lib.svs_init.restype = ctypes.c_int
        lib.svs_release.argtypes = [P]
        lib.svs_release.restype = None
        lib.svs_last_error.argtypes = []
        lib.svs_last_error.restype = ctypes.c_char_p
        lib.svs_device_count.argtypes = [ctypes.POINTER(ctypes.c_int)]
        lib.svs_device_count.restype = ctypes.c_int
        lib.svs_poa_batch.argtypes = [P, I32, ctypes.POINTER(I64), ctypes.POINTER(I64), ctypes.c_char_p,
                                      ctypes.POINTER(PoaConfig), ctypes.POINTER(P)]
        lib.svs_poa_batch.restype = ctypes.c_int
        lib.svs_poa_result_consensus.argtypes = [P, I32, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(I64)]
        lib.svs_poa_result_consensus.restype = ctypes.c_int
        lib.svs_poa_result_msa.argtypes = [P, I32, ctypes.POINTER(I32), ctypes.POINTER(I32),
                                           ctypes.POINTER(ctypes.c_void_p)]
        lib.svs_poa_result_msa.restype = ctypes.c_int
        lib.svs_poa_result_stats.argtypes = [P, ctypes.POINTER(PoaStats)]
        lib.svs_poa_result_stats.restype = ctypes.c_int
        lib.svs_poa_result_free.argtypes = [P]
        lib.svs_poa_result_free.restype = None
        lib.svs_wave_selftest.argtypes = [P, P, P, P, I32]
        lib.svs_wave_selftest.restype = ctypes.c_int
        _declare_em(lib)
        _lib = lib
        return lib


def _declare_em(lib):
    if not hasattr(lib, "svs_em_batch"):
        return
    P, I32 = ctypes.c_void_p, ctypes.c_int32
    lib.svs_rng_exponential_table.argtypes = [ctypes.c_uint32, ctypes.c_int64, P]
    lib.svs_rng_exponential_table.restype = ctypes.c_int
    lib.svs_similarity_batch.argtypes = [P, I32, ctypes.POINTER(EmWindow), P, P, P]
    lib.svs_similarity_batch.restype = ctypes.c_int
    lib.svs_em_batch.argtypes = [P, I32, ctypes.POINTER(EmWindow), P, P, ctypes.POINTER(EmConfig),
                                 ctypes.POINTER(ctypes.c_void_p)]
    lib.svs_em_batch.restype = ctypes.c_int
    lib.svs_ward_maxclust_batch.argtypes = [I32, ctypes.POINTER(EmWindow), P, P, I32, P]
    lib.svs_ward_maxclust_batch.restype = ctypes.c_int
    lib.svs_em_cluster_batch.argtypes = [P, I32, ctypes.POINTER(EmWindow), P, ctypes.POINTER(EmConfig),
                                         ctypes.POINTER(ctypes.c_void_p)]
    lib.svs_em_cluster_batch.restype = ctypes.c_int
    lib.svs_decision_batch.argtypes = [P, I32, ctypes.POINTER(DecisionWindow), P, P, P, P,
                                       ctypes.POINTER(DecisionConfig), ctypes.POINTER(ctypes.c_void_p)]
    lib.svs_decision_batch.restype = ctypes.c_int
    PI32 = ctypes.POINTER(ctypes.c_int32)
    lib.svs_decision_session_open.argtypes = [P, ctypes.POINTER(DecisionConfig), ctypes.POINTER(ctypes.c_void_p)]
    lib.svs_decision_session_open.restype = ctypes.c_int
    lib.svs_decision_session_submit.argtypes = [P, I32, ctypes.POINTER(DecisionWindow), P, P, P, P,
                                                ctypes.POINTER(ctypes.c_int64)]
    lib.svs_decision_session_submit.restype = ctypes.c_int
    lib.svs_decision_session_wait.argtypes = [P, ctypes.c_int64, ctypes.POINTER(ctypes.c_void_p)]
    lib.svs_decision_session_wait.restype = ctypes.c_int
    lib.svs_decision_session_stats.argtypes = [P, ctypes.POINTER(DecisionStats)]
    lib.svs_decision_session_stats.restype = ctypes.c_int
    lib.svs_decision_session_close.argtypes = [P]
    lib.svs_decision_session_close.restype = ctypes.c_int
    lib.svs_decision_result_window.argtypes = [P, I32, PI32, PI32, PI32, PI32]
    lib.svs_decision_result_window.restype = ctypes.c_int
    lib.svs_decision_result_window_error.argtypes = [P, I32, ctypes.POINTER(ctypes.c_char_p)]
    lib.svs_decision_result_window_error.restype = ctypes.c_int
    lib.svs_decision_result_cluster.argtypes = [P, I32, I32, ctypes.POINTER(PI32), PI32,
                                                ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_int64)]
    lib.svs_decision_result_cluster.restype = ctypes.c_int
    lib.svs_decision_result_stats.argtypes = [P, ctypes.POINTER(DecisionStats)]
    lib.svs_decision_result_stats.restype = ctypes.c_int
    lib.svs_decision_result_free.argtypes = [P]
    lib.svs_decision_result_free.restype = None
    lib.svs_msa_features.argtypes = [I32, I32, P, P, I32, P, I32, I32, P, I32, I32, ctypes.c_double, PI32, PI32,
                                     P, ctypes.c_int64, P, PI32, ctypes.c_int64]
    lib.svs_msa_features.restype = ctypes.c_int
    lib.svs_em_result_get.argtypes = [P, I32, I32, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_int64)]
    lib.svs_em_result_get.restype = ctypes.c_int
    lib.svs_em_result_stats.argtypes = [P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64)]
    lib.svs_em_result_stats.restype = ctypes.c_int
    lib.svs_em_result_free.argtypes = [P]
    lib.svs_em_result_free.restype = None
    lib.svs_aligment_score_batch.argtypes = [P, I32, P, P, I32, P, P, I32, P, P, P, ctypes.POINTER(MisscoreStats)]
    lib.svs_aligment_score_batch.restype = ctypes.c_int


def check(rc, what="svscope call"):
    if rc != SVS_OK:
        msg = load_library().svs_last_error()
        raise SvsError(f"{what} failed ({_ERRNAMES.get(rc, rc)}): {msg.decode() if msg else ''}")


class Context:
    """One HIP stream + device arenas (C++ svs_context)."""

    def __init__(self, device=0):
        self.lib = load_library()
        h = ctypes.c_void_p()
        check(self.lib.svs_init(int(device), ctypes.byref(h)), "svs_init")
        self.handle = h
        self.device = device

    def close(self):
        if getattr(self, "handle", None):
            self.lib.svs_release(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_contexts = {}
_ctx_lock = threading.Lock()


def default_context(device=None):
    """Process-wide context per device (ctypes calls are serialised by the caller)."""
    if device is None:
        device = int(os.environ.get("SVS_DEVICE", "0"))
    with _ctx_lock:
        ctx = _contexts.get(device)
        if ctx is None:
            ctx = Context(device)
            _contexts[device] = ctx
        return ctx
