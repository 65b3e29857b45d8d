"""ctypes binding of libcwq.so (the C ABI in include/cwq.h).

The product path has exactly one implementation: the gfx950 HIP kernels in
``csrc/``.  If the library is missing or cannot be loaded this module raises;
there is no CPU fallback.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# CWQ_LIB_PATH selects another build of the same library (tools/variants.sh
# A/B-times compile-time tuning variants this way); default is the in-tree one.
LIB_PATH = os.environ.get("CWQ_LIB_PATH") or os.path.join(_HERE, "libcwq.so")

c_int = ctypes.c_int
c_i32 = ctypes.c_int32
c_i64 = ctypes.c_int64
c_f32 = ctypes.c_float
c_f64 = ctypes.c_double
c_size = ctypes.c_size_t
c_vp = ctypes.c_void_p
c_str = ctypes.c_char_p


class Options(ctypes.Structure):
    """cwq_options (include/cwq.h): per-call encoder options."""
    _fields_ = [("prune_mode", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("eval_start_event", c_vp), ("eval_stop_event", c_vp),
                ("eval_ms_out", ctypes.POINTER(ctypes.c_float)),
                ("item_ready", c_vp)]


c_opts = ctypes.POINTER(Options)


def options(prune_mode=None, eval_events=None, eval_ms_out=None, item_ready=None):
    """A cwq_options pointer for one call, or None (the library defaults:
    prune_mode 2, no events).  eval_events: (start, stop) hipEvent_t handles;
    eval_ms_out: a ctypes.c_float the fused grouped calls write their scoring
    launches' milliseconds to; item_ready: the address of the batch call's
    per-item int32 flags (zeroed)."""
    if prune_mode is None and eval_events is None and eval_ms_out is None and item_ready is None:
        return None
    o = Options(2 if prune_mode is None else int(prune_mode), 0, None, None, None, item_ready)
    if eval_events is not None:
        o.eval_start_event, o.eval_stop_event = eval_events
    if eval_ms_out is not None:
        o.eval_ms_out = ctypes.pointer(eval_ms_out)
    return ctypes.pointer(o)


# name -> (restype, argtypes); mirrors include/cwq.h one-to-one.
SIGNATURES = {
    "cwq_version": (c_int, []),
    "cwq_last_error": (c_str, []),
    "cwq_stateless_normal_sample": (c_int, [c_vp, c_vp, c_i64, c_i64, c_i32, c_vp, c_vp]),
    "cwq_greedy_encode_workspace_size": (c_size, [c_i64, c_i64, c_i64]),
    "cwq_greedy_encode_uniform_workspace_size": (c_size, [c_i64, c_i64]),
    "cwq_greedy_encode": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_int,
                                  c_int, c_i32, c_f32, c_i64, c_vp, c_vp, c_vp, c_size, c_opts,
                                  c_vp]),
    "cwq_greedy_encode_uniform": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_int, c_int,
                                          c_i32, c_f32, c_i64, c_vp, c_vp, c_vp, c_size, c_opts,
                                          c_vp]),
    "cwq_greedy_decode": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_int, c_int,
                                  c_i32, c_f32, c_i64, c_vp, c_vp]),
    "cwq_greedy_decode_uniform": (c_int, [c_vp, c_vp, c_vp, c_i64, c_i64, c_int, c_int, c_i32,
                                          c_f32, c_i64, c_vp, c_vp]),
    "cwq_standardise": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp]),
    "cwq_kl_normal_normal": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp]),
    "cwq_destandardise": (c_int, [c_vp, c_vp, c_vp, c_i64, c_vp, c_vp]),
    "cwq_group_starts": (c_i64, [c_vp, c_i64, c_i64, c_f64, c_vp, c_i64]),
    "cwq_code_grouped_greedy_workspace_size": (c_size, [c_i64, c_int]),
    "cwq_code_grouped_greedy": (c_i64, [c_vp, c_vp, c_vp, c_vp, c_i64, c_int, c_int, c_i32, c_f32,
                                        c_i64, c_f64, c_vp, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp,
                                        c_size, c_opts, c_vp]),
    "cwq_code_grouped_greedy_begin": (c_i64, [c_vp, c_vp, c_vp, c_vp, c_i64, c_int, c_int, c_i32,
                                              c_f32, c_i64, c_f64, c_vp, c_vp, c_i64, c_vp, c_i64,
                                              c_vp, c_vp, c_size, c_opts, c_vp]),
    "cwq_code_grouped_greedy_end": (c_i64, [c_vp, c_i64, c_int, c_int, c_vp, c_i64, c_vp]),
    "cwq_code_grouped_greedy_batch_workspace_size": (c_size, [c_i64, c_i64, c_int]),
    "cwq_code_grouped_greedy_batch_host_workspace_size": (c_size, [c_i64, c_i64, c_int]),
    "cwq_code_grouped_greedy_batch": (c_i64, [c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int,
                                              c_vp, c_f32, c_i64, c_f64, c_vp, c_vp, c_i64, c_vp,
                                              c_vp, c_i64, c_vp, c_vp, c_size, c_vp, c_size,
                                              c_opts, c_vp]),
    "cwq_importance_workspace_size": (c_size, [c_i64, c_i64]),
    "cwq_importance_encode": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i32,
                                      c_i64, c_vp, c_vp, c_vp, c_size, c_opts, c_vp]),
    "cwq_importance_decode": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i32, c_i64, c_vp,
                                      c_vp]),
    "cwq_importance_group_starts": (c_i64, [c_vp, c_i64, c_i64, c_f64, c_vp, c_i64]),
    "cwq_importance_plan": (c_int, [c_vp, c_vp, c_i64, c_vp]),
    "cwq_code_grouped_importance_workspace_size": (c_size, [c_i64]),
    "cwq_code_grouped_importance": (c_i64, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_f32, c_i64,
                                            c_f64, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp,
                                            c_vp, c_vp, c_size, c_opts, c_vp]),
    "cwq_code_grouped_importance_batch_workspace_size": (c_size, [c_i64, c_i64]),
    "cwq_code_grouped_importance_batch": (c_i64, [c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                                  c_f32, c_i64, c_f64, c_vp, c_vp, c_vp, c_i64,
                                                  c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_size,
                                                  c_opts, c_vp]),
    "cwq_ac_encode": (c_i64, [c_vp, c_i64, c_int, c_vp, c_i64, c_vp, c_i64]),
    "cwq_ac_decode": (c_i64, [c_vp, c_i64, c_int, c_vp, c_i64, c_vp, c_i64]),
    "cwq_elias_delta_encode": (c_i64, [c_vp, c_i64, c_vp, c_i64]),
    "cwq_elias_delta_decode": (c_i64, [c_vp, c_i64, c_i64, c_vp]),
    "cwq_bitcode_to_indices": (c_i64, [c_vp, c_i64, c_int, c_i64, c_vp]),
    "cwq_selftest_bm_tables": (c_int, [ctypes.c_uint32, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "cwq_selftest_screen_tables": (c_int, [ctypes.c_uint32, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "cwq_selftest_logf": (c_int, [c_vp, c_i64, c_vp, c_vp]),
    "cwq_selftest_wave_max": (c_int, [c_vp, c_i64, c_vp, c_vp]),
    "cwq_selftest_div": (c_int, [c_vp, c_vp, c_i64, c_vp, c_vp]),
    "cwq_pln_posterior": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_f32, c_vp, c_vp, c_vp]),
    "cwq_permute_gather": (c_int, [c_vp, c_i64, c_i64, c_vp, c_vp, c_vp]),
    "cwq_permute_scatter": (c_int, [c_vp, c_i64, c_i64, c_vp, c_vp, c_vp]),
}

# Tools-only entry points (csrc/cwq_debug.h, not in include/cwq.h).
TOOL_SIGNATURES = {
    "cwq_debug_prune_stats": (c_int, [c_vp, c_int]),
    "cwq_debug_tile_times": (c_int, [c_vp, c_vp, c_vp, c_int]),
    "cwq_debug_quad_times": (c_int, [c_vp, c_vp, c_int]),
    "cwq_debug_partition_workspace_size": (c_size, [c_i64]),
    "cwq_debug_group_starts_device": (c_i64, [c_vp, c_i64, c_i64, c_f64, c_vp, c_vp, c_size,
                                              c_vp, c_vp]),
}

# CWQ_ABI_VERSION of the include/cwq.h these signatures mirror: a library
# reporting another version has other argument lists and is refused.
ABI_VERSION = (0 << 16) | 6

_lib = None


class CwqError(RuntimeError):
    """A libcwq call returned an error code."""


def load():
    """Load libcwq.so (once).  Raises if it is absent: no fallback exists."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} not found: build the HIP extension first "
            "(python -c 'import __graft_entry__ as g; g.build()')")
    lib = ctypes.CDLL(LIB_PATH)
    lib.cwq_version.restype = c_int
    lib.cwq_version.argtypes = []
    ver = lib.cwq_version()
    if ver != ABI_VERSION:
        raise ImportError(f"{LIB_PATH} has ABI version {ver >> 16}.{ver & 0xffff}, these "
                          f"bindings need {ABI_VERSION >> 16}.{ABI_VERSION & 0xffff}: rebuild it")
    for name, (res, args) in list(SIGNATURES.items()) + list(TOOL_SIGNATURES.items()):
        if not hasattr(lib, name):
            if name in TOOL_SIGNATURES:  # tools only: a product build need not export them
                continue
            raise ImportError(f"{LIB_PATH} does not export {name}: rebuild it")
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc, what):
    if rc < 0:
        msg = load().cwq_last_error().decode("utf-8", "replace")
        raise CwqError(f"{what} failed ({rc}): {msg}")
    return rc
