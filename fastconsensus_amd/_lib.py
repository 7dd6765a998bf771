"""ctypes binding of libfastconsensus_amd.so (C-ABI: include/fastconsensus_amd.h).

The product path has NO CPU fallback: if the library is missing or no gfx950 device is
visible, every engine call raises.
"""
import ctypes
import os

import numpy as np

PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FC_LIB_PATH") or os.path.join(PKG, "lib", "libfastconsensus_amd.so")

FC_ALGO_LOUVAIN = 0
FC_ALGO_LPM = 1
FC_ALGO_LOUVAIN_NC = 2   # louvain with new_consensus.py's weight rule (:155-163)
FC_ALGO_LEIDEN = 3       # leiden branch (:204-258, final pass :385-388)
FC_ALGO_INFOMAP = 4      # infomap: the lpm loop (:260-310) around igraph Infomap (:268, :390)
OPTIONS = {"buckets": 1, "max_sweeps": 2, "max_iters": 3, "chunk": 4, "prune": 5, "relabel": 6, "tail_visits": 7,
           "coarsen": 8, "store": 9, "seed": 10, "closure_rounds": 11,
           "prune_mark": 12, "infomap_trials": 13, "cd_engine": 14,
           "rl_min_replicas": 15, "rl_min_vertices": 16, "dense_div": 17}
ERRORS = {-1: "EINVAL", -2: "ENODEV", -3: "EHIP", -4: "ESTATE", -5: "ELIMIT"}

# Every symbol declared in include/fastconsensus_amd.h (checked by tests/test_capi_symbols.py)
SYMBOLS = [
    "fc_last_error", "fc_version", "fc_build_hash", "fc_create", "fc_destroy", "fc_set_stream", "fc_synchronize", "fc_set_timing",
    "fc_collect_timing", "fc_set_params", "fc_set_option", "fc_load_graph", "fc_graph_info", "fc_get_node_map", "fc_reset_graph", "fc_get_graph", "fc_get_nextgraph", "fc_run",
    "fc_cd", "fc_set_labels", "fc_replica_info", "fc_get_labels", "fc_consensus_partial", "fc_consensus_apply",
    "fc_closure_sample", "fc_closure_set_pairs", "fc_closure_begin", "fc_closure_block_sample",
    "fc_closure_block_add", "fc_closure_finish", "fc_closure_partial", "fc_closure_apply",
    "fc_generate_lfr", "fc_generate_sbm", "fc_read_edgelist",
]


class FastConsensusError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("%s (%s): %s" % (ERRORS.get(code, code), code, msg))
        self.code = code


class Stats(ctypes.Structure):
    _fields_ = [
        ("iterations", ctypes.c_int32), ("exit_check", ctypes.c_int32), ("hit_iter_cap", ctypes.c_int32),
        ("n_p", ctypes.c_int32), ("m_final", ctypes.c_int64), ("partition_edges", ctypes.c_int64),
        ("cd_sweeps", ctypes.c_int64), ("cd_vertex_visits", ctypes.c_int64), ("cd_edge_visits", ctypes.c_int64),
        ("cd_ms", ctypes.c_double), ("consensus_ms", ctypes.c_double), ("closure_ms", ctypes.c_double),
        ("rebuild_ms", ctypes.c_double), ("decide_ms", ctypes.c_double), ("decide_launches", ctypes.c_int64),
        ("decide_bytes", ctypes.c_int64),
        ("lv_decide_ms", ctypes.c_double), ("lv_decide_launches", ctypes.c_int64), ("lv_decide_bytes", ctypes.c_int64),
        ("lv_heavy_ms", ctypes.c_double), ("lv_heavy_launches", ctypes.c_int64), ("lv_heavy_bytes", ctypes.c_int64),
        ("rl_decide_ms", ctypes.c_double), ("rl_decide_launches", ctypes.c_int64), ("rl_decide_bytes", ctypes.c_int64),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


_lib = None
_i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
_i64p = np.ctypeslib.ndpointer(np.int64, flags="C_CONTIGUOUS")


def load():
    """Load the native library (raises if it was not built: no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise FastConsensusError(-2, "native library %s not built; run `python -m fastconsensus_amd.build`"
                                 % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH)
    c_int, i32, i64, u64, dbl, vp = ctypes.c_int, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, \
        ctypes.c_double, ctypes.c_void_p
    P = ctypes.POINTER
    L.fc_last_error.restype = ctypes.c_char_p
    L.fc_version.restype = ctypes.c_char_p
    L.fc_build_hash.restype = ctypes.c_char_p
    L.fc_create.argtypes = [c_int, u64, P(vp)]
    L.fc_destroy.argtypes = [vp]
    L.fc_destroy.restype = None
    L.fc_set_stream.argtypes = [vp, vp]
    L.fc_synchronize.argtypes = [vp]
    L.fc_set_timing.argtypes = [vp, c_int]
    L.fc_collect_timing.argtypes = [vp, P(Stats)]
    L.fc_set_params.argtypes = [vp, c_int, c_int, c_int]
    L.fc_set_option.argtypes = [vp, c_int, i64]
    L.fc_load_graph.argtypes = [vp, i64, i64, _i32p, _i32p]
    L.fc_reset_graph.argtypes = [vp]
    L.fc_get_node_map.argtypes = [vp, _i32p]
    L.fc_graph_info.argtypes = [vp, P(i64), P(i64), P(i64)]
    L.fc_get_graph.argtypes = [vp, vp, vp, vp, vp]
    L.fc_get_nextgraph.argtypes = [vp, P(i64), vp, vp, vp, vp]
    L.fc_run.argtypes = [vp, c_int, c_int, dbl, dbl, vp, P(Stats)]
    L.fc_cd.argtypes = [vp, c_int, c_int, c_int, c_int, c_int]
    L.fc_set_labels.argtypes = [vp, c_int, _i32p]
    L.fc_replica_info.argtypes = [vp, P(c_int), P(c_int), P(c_int)]
    L.fc_get_labels.argtypes = [vp, vp, i64, c_int]   # host array or device buffer, capacity
    L.fc_consensus_partial.argtypes = [vp, c_int, vp]
    L.fc_consensus_apply.argtypes = [vp, c_int, c_int, dbl, dbl, vp, P(c_int), P(i64), P(i64)]
    L.fc_closure_sample.argtypes = [vp, i64, c_int, P(i64)]
    L.fc_closure_set_pairs.argtypes = [vp, i64, vp, c_int, P(i64)]
    L.fc_closure_begin.argtypes = [vp, i64, c_int, P(c_int)]
    L.fc_closure_block_sample.argtypes = [vp, c_int, i64, i64, vp, i64, P(i64)]
    L.fc_closure_block_add.argtypes = [vp, c_int, vp, i64]
    L.fc_closure_finish.argtypes = [vp, P(i64)]
    L.fc_closure_partial.argtypes = [vp, vp]
    L.fc_closure_apply.argtypes = [vp, c_int, c_int, dbl, vp, c_int, P(c_int), P(i64)]
    L.fc_generate_lfr.argtypes = [i64, dbl, dbl, dbl, dbl, i32, i32, i32, u64, i64, vp, vp, P(i64), vp]
    L.fc_generate_sbm.argtypes = [i64, i32, dbl, dbl, u64, i64, vp, vp, P(i64)]
    L.fc_read_edgelist.argtypes = [ctypes.c_char_p, P(i64), P(i64), vp, vp, vp]
    _lib = L
    return L


def check(rc):
    if rc != 0:
        raise FastConsensusError(rc, load().fc_last_error().decode(errors="replace"))
    return rc


def ptr(a):
    """Raw address of a numpy array, a torch tensor, or an int (None -> NULL)."""
    if a is None:
        return None
    if isinstance(a, int):
        return a
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    if hasattr(a, "data_ptr"):
        return a.data_ptr()
    raise TypeError("cannot take the address of %r" % type(a))
