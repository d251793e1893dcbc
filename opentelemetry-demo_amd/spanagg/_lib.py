"""ctypes binding of libspanagg's C-ABI (include/spanagg.h).

The shared library is built in-tree (``make -C opentelemetry-demo_amd``) next to
this file.  There is no fallback: if the library is missing, ``load()`` raises,
and if no gfx950 device is present ``sa_create`` fails with SA_EDEVICE.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# SPANAGG_LIB: another build of the same ABI -- libspanagg_ab.so, the laboratory
# build tools/ use for A/B variants and ablations (`make -C opentelemetry-demo_amd ab`)
LIB_PATH = os.environ.get("SPANAGG_LIB") or os.path.join(_HERE, "libspanagg.so")

SA_OK, SA_EINVAL, SA_ENOMEM, SA_EDEVICE, SA_EFULL, SA_ERANGE, SA_ESTATE = 0, -1, -2, -3, -4, -5, -6
SA_UNIT_MS, SA_UNIT_S = 0, 1
SA_MAX_BOUNDS = 62
# sa_config.options (include/spanagg.h SA_OPT_*): alternative kernel paths with
# the same results, for parity tests and A/B runs
OPT_NO_HLL_FILTER, OPT_PARTITIONED, OPT_ATOMIC_TABLE, OPT_EXPO_HBM, OPT_EXPO_CACHED = 1, 2, 4, 8, 16
OPT_IDENTITY_IDS, OPT_STAMPS, OPT_GROUP_COPY, OPT_GROUP_RCCL = 32, 64, 128, 256
STATUS_NAMES = {
    SA_OK: "SA_OK", SA_EINVAL: "SA_EINVAL", SA_ENOMEM: "SA_ENOMEM", SA_EDEVICE: "SA_EDEVICE",
    SA_EFULL: "SA_EFULL", SA_ERANGE: "SA_ERANGE", SA_ESTATE: "SA_ESTATE",
}

u64p = C.POINTER(C.c_uint64)
u32p = C.POINTER(C.c_uint32)
u8p = C.POINTER(C.c_uint8)
f64p = C.POINTER(C.c_double)


class sa_config(C.Structure):
    _fields_ = [
        ("bounds", f64p), ("n_bounds", C.c_uint32), ("unit", C.c_uint32),
        ("hll_p", C.c_uint32), ("cms_d", C.c_uint32), ("cms_w", C.c_uint32),
        ("window_ns", C.c_uint64), ("n_windows", C.c_uint32), ("n_services", C.c_uint32),
        ("key_capacity", C.c_uint64), ("device", C.c_int32), ("flags", C.c_uint32),
        ("exp_max_size", C.c_uint32), ("options", C.c_uint32),
    ]


class sa_span_batch(C.Structure):
    _fields_ = [
        ("key_hash", C.c_void_p), ("start_ns", C.c_void_p), ("end_ns", C.c_void_p),
        ("trace_w0", C.c_void_p), ("trace_w1", C.c_void_p), ("meta", C.c_void_p),
        ("n", C.c_uint64),
    ]


class sa_red_result(C.Structure):
    _fields_ = [
        ("n_series", C.c_uint64), ("n_buckets", C.c_uint32),
        ("key_hash", u64p), ("bucket_counts", u64p), ("calls", u64p),
        ("sum_ns", u64p), ("sum", f64p),
    ]


class sa_exp_result(C.Structure):
    _fields_ = [
        ("n_series", C.c_uint64), ("max_size", C.c_uint32), ("unit", C.c_uint32),
        ("key_hash", u64p), ("count", u64p), ("zero_count", u64p), ("sum_ns", u64p),
        ("sum", f64p), ("min", f64p), ("max", f64p),
        ("scale", C.POINTER(C.c_int32)), ("offset", C.POINTER(C.c_int32)), ("n_buckets", u32p),
        ("bucket_counts", u64p),
    ]


class sa_sketch_result(C.Structure):
    _fields_ = [
        ("window_id", C.c_uint64), ("n_services", C.c_uint32), ("hll_p", C.c_uint32),
        ("hll", u8p), ("cms_d", C.c_uint32), ("cms_w", C.c_uint32), ("cms", u32p),
    ]


class sa_stats(C.Structure):
    _fields_ = [
        ("spans", C.c_uint64), ("zero_key", C.c_uint64), ("invalid_service", C.c_uint64),
        ("window_out_of_range", C.c_uint64), ("dropped_table_full", C.c_uint64),
        ("n_keys", C.c_uint64), ("table_capacity", C.c_uint64), ("window_base", C.c_uint64),
        ("small_table", C.c_uint32), ("pad", C.c_uint32), ("hll_filtered", C.c_uint64),
    ]


# (name, restype, argtypes) for every entry point declared in include/spanagg.h
SIGNATURES = [
    ("sa_config_default", None, [C.POINTER(sa_config)]),
    ("sa_abi_version", C.c_int, []),
    ("sa_create", C.c_int, [C.POINTER(sa_config), C.POINTER(C.c_void_p)]),
    ("sa_destroy", None, [C.c_void_p]),
    ("sa_last_error", C.c_char_p, [C.c_void_p]),
    ("sa_ingest", C.c_int, [C.c_void_p, C.POINTER(sa_span_batch)]),
    ("sa_ingest_async", C.c_int, [C.c_void_p, C.POINTER(sa_span_batch)]),
    ("sa_ingest_device", C.c_int, [C.c_void_p, C.POINTER(sa_span_batch), C.c_void_p]),
    ("sa_ingest_device_many", C.c_int, [C.c_void_p, C.POINTER(sa_span_batch), C.c_uint32, C.c_void_p]),
    ("sa_host_alloc", C.c_int, [C.c_size_t, C.POINTER(C.c_void_p)]),
    ("sa_host_free", None, [C.c_void_p]),
    ("sa_sync", C.c_int, [C.c_void_p]),
    ("sa_flush", C.c_int, [C.c_void_p, C.POINTER(C.POINTER(sa_red_result))]),
    ("sa_red_result_free", None, [C.POINTER(sa_red_result)]),
    ("sa_flush_exp", C.c_int, [C.c_void_p, C.POINTER(C.POINTER(sa_exp_result))]),
    ("sa_reclaim_keys", C.c_int, [C.c_void_p, C.c_int]),
    ("sa_exp_result_free", None, [C.POINTER(sa_exp_result)]),
    ("sa_expo_probe", C.c_int, [C.c_void_p, f64p, C.POINTER(C.c_int32), C.c_uint64, C.POINTER(C.c_int32), f64p]),
    ("sa_key_union_probe", C.c_int, [C.c_void_p, u64p, C.c_uint64, u64p, u64p]),
    ("sa_join", C.c_int, [C.c_void_p, C.c_void_p]),
    ("sa_expo_fast_probe", C.c_int, [C.c_void_p, u64p, C.POINTER(C.c_int32), C.c_uint64, C.POINTER(C.c_int32),
                                     C.POINTER(C.c_int32), f64p]),
    ("sa_window_read", C.c_int, [C.c_void_p, C.c_uint64, C.POINTER(C.POINTER(sa_sketch_result))]),
    ("sa_window_advance", C.c_int, [C.c_void_p, C.c_uint64]),
    ("sa_sketch_result_free", None, [C.POINTER(sa_sketch_result)]),
    ("sa_get_stats", C.c_int, [C.c_void_p, C.POINTER(sa_stats)]),
    ("sa_export_keys", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, u64p, C.c_void_p]),
    ("sa_gather_dense", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_int, C.c_void_p]),
    ("sa_window_export", C.c_int, [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p]),
    ("sa_group_create", C.c_int, [C.POINTER(sa_config), C.POINTER(C.c_int32), C.c_uint32,
                                  C.POINTER(C.c_void_p)]),
    ("sa_group_destroy", None, [C.c_void_p]),
    ("sa_group_last_error", C.c_char_p, [C.c_void_p]),
    ("sa_group_size", C.c_uint32, [C.c_void_p]),
    ("sa_group_uses_rccl", C.c_int, [C.c_void_p]),
    ("sa_group_member", C.c_void_p, [C.c_void_p, C.c_uint32]),
    ("sa_group_ingest", C.c_int, [C.c_void_p, C.POINTER(sa_span_batch)]),
    ("sa_group_ingest_device", C.c_int, [C.c_void_p, C.POINTER(sa_span_batch), C.c_uint32, C.c_void_p]),
    ("sa_group_sync", C.c_int, [C.c_void_p]),
    ("sa_group_flush", C.c_int, [C.c_void_p, C.POINTER(C.POINTER(sa_red_result))]),
    ("sa_group_flush_exp", C.c_int, [C.c_void_p, C.POINTER(C.POINTER(sa_exp_result))]),
    ("sa_group_window_read", C.c_int, [C.c_void_p, C.c_uint64, C.POINTER(C.POINTER(sa_sketch_result))]),
    ("sa_group_window_advance", C.c_int, [C.c_void_p, C.c_uint64]),
    ("sa_group_get_stats", C.c_int, [C.c_void_p, C.POINTER(sa_stats)]),
    ("sa_debug_stamps", C.c_int, [C.c_void_p, u64p, C.c_uint64, u64p]),
    ("sa_bucket_thresholds", C.c_int, [f64p, C.c_uint32, C.c_uint32, u64p, u32p]),
    ("sa_hll_estimate", C.c_double, [u8p, C.c_uint32]),
]

ABI_VERSION = 4  # include/spanagg.h SA_ABI_VERSION

_lib = None


def load() -> C.CDLL:
    """Load libspanagg.so (in-tree build). Raises if it was not built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"libspanagg.so not found at {LIB_PATH}; build it with "
                "`make -C opentelemetry-demo_amd` (or __graft_entry__.build())")
        # torch ships its own libamdhip64.so.7. Loading torch first makes
        # libspanagg bind to that same HIP runtime (same soname), so device
        # pointers and streams are shared; loading /opt/rocm's copy first
        # leaves torch with a second runtime that sees no GPUs.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        lib = C.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            fn = getattr(lib, name, None)
            if fn is None and os.environ.get("SPANAGG_LIB"):
                continue  # an older diagnostic build may lack newer entry points
            if fn is None:
                raise RuntimeError(f"libspanagg.so does not export {name}")
            fn.restype = res
            fn.argtypes = args
        if lib.sa_abi_version() != ABI_VERSION:
            raise RuntimeError("libspanagg ABI version mismatch")
        _lib = lib
    return _lib


class SpanAggError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{STATUS_NAMES.get(code, code)}: {msg}")
        self.code = code
