"""Python host wrapper of one libspanagg engine (one engine per GPU / rank).

Maps the connector's lifecycle onto the C-ABI:
``Engine(config)`` ~ createTracesToMetricsConnector + Start, ``ingest`` ~ the
per-span body of ConsumeTraces, ``flush`` ~ exportMetrics' buildMetrics +
resetState (delta since the previous flush), ``close`` ~ Shutdown.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import Optional, Sequence

import numpy as np

from . import _lib
from ._lib import SpanAggError

DEFAULT_BOUNDS_MS = (2, 4, 6, 8, 10, 50, 100, 200, 400, 800, 1000, 1400, 2000, 5000, 10000, 15000)

KIND_SHIFT, STATUS_SHIFT = 16, 19


def pack_meta(service_id, kind, status) -> np.ndarray:
    """meta = service_id | kind << 16 | status << 19 (SoA v1)."""
    s = np.asarray(service_id, dtype=np.uint32)
    k = np.asarray(kind, dtype=np.uint32)
    c = np.asarray(status, dtype=np.uint32)
    if np.any(s > 0xFFFF) or np.any(k > 7) or np.any(c > 3):
        raise ValueError("meta field out of range")
    return (s | (k << KIND_SHIFT) | (c << STATUS_SHIFT)).astype(np.uint32)


def trace_words(trace_ids: np.ndarray):
    """[n,16] u8 wire trace ids -> (w0, w1) little-endian u64 words."""
    t = np.ascontiguousarray(trace_ids, dtype=np.uint8).reshape(-1, 16)
    w = t.view("<u8").reshape(-1, 2)
    return np.ascontiguousarray(w[:, 0]), np.ascontiguousarray(w[:, 1])


@dataclass
class Config:
    """Mirror of the spanmetrics Config fields this engine consumes plus the
    build-owned sketch parameters (defaults = the reference's empty
    `spanmetrics:` block, otelcol-config.yml:115-116)."""
    bounds: Sequence[float] = DEFAULT_BOUNDS_MS
    unit: str = "ms"
    hll_p: int = 14
    cms_d: int = 4
    cms_w: int = 2048
    window_ns: int = 10_000_000_000
    n_windows: int = 8
    n_services: int = 64
    key_capacity: int = 1000
    device: int = 0
    flags: int = 0  # SA_DIAG_* profiling ablations only (laboratory build; results are wrong when set)
    exp_max_size: int = 0  # histogram.exponential.max_size (0: explicit buckets)
    options: int = 0  # SA_OPT_* path options (spanagg._lib.OPT_*): same results, another kernel path

    def to_c(self):
        arr = (C.c_double * max(1, len(self.bounds)))(*[float(b) for b in self.bounds])
        c = _lib.sa_config()
        c.bounds = C.cast(arr, _lib.f64p)
        c.n_bounds = len(self.bounds)
        c.unit = _lib.SA_UNIT_S if self.unit == "s" else _lib.SA_UNIT_MS
        c.hll_p, c.cms_d, c.cms_w = self.hll_p, self.cms_d, self.cms_w
        c.window_ns, c.n_windows, c.n_services = self.window_ns, self.n_windows, self.n_services
        c.key_capacity, c.device, c.flags = self.key_capacity, self.device, self.flags
        c.exp_max_size, c.options = self.exp_max_size, self.options
        return c, arr


@dataclass
class SpanBatch:
    key_hash: np.ndarray
    start_ns: np.ndarray
    end_ns: np.ndarray
    trace_w0: np.ndarray
    trace_w1: np.ndarray
    meta: np.ndarray

    def __post_init__(self):
        for name in ("key_hash", "start_ns", "end_ns", "trace_w0", "trace_w1"):
            setattr(self, name, np.ascontiguousarray(getattr(self, name), dtype=np.uint64))
        self.meta = np.ascontiguousarray(self.meta, dtype=np.uint32)
        n = len(self.key_hash)
        if any(len(getattr(self, f)) != n for f in
               ("start_ns", "end_ns", "trace_w0", "trace_w1", "meta")):
            raise ValueError("ragged SoA batch")

    def __len__(self):
        return len(self.key_hash)

    def slice(self, a: int, b: int) -> "SpanBatch":
        return SpanBatch(self.key_hash[a:b], self.start_ns[a:b], self.end_ns[a:b],
                         self.trace_w0[a:b], self.trace_w1[a:b], self.meta[a:b])

    def columns(self):
        return (self.key_hash, self.start_ns, self.end_ns, self.trace_w0, self.trace_w1, self.meta)


@dataclass
class RedResult:
    key_hash: np.ndarray          # [n] u64, ascending
    bucket_counts: np.ndarray     # [n, n_buckets] u64
    calls: np.ndarray             # [n] u64
    sum_ns: np.ndarray            # [n] u64
    sum: np.ndarray               # [n] f64 (ms or s)
    status: int = 0


@dataclass
class ExpoResult:
    """sa_exp_result: per series go-expohisto histograms (delta since the last flush)."""
    key_hash: np.ndarray     # [n] u64, ascending
    count: np.ndarray        # [n] u64
    zero_count: np.ndarray   # [n] u64
    sum_ns: np.ndarray       # [n] u64
    sum: np.ndarray          # [n] f64 (unit)
    min: np.ndarray
    max: np.ndarray
    scale: np.ndarray        # [n] i32
    offset: np.ndarray       # [n] i32
    buckets: list            # [n] u64 arrays (positive buckets offset .. offset + len - 1)
    status: int = 0


@dataclass
class SketchResult:
    window_id: int
    hll: np.ndarray               # [n_services, 2^p] u8
    cms: np.ndarray               # [d, w] u32
    p: int = 14

    def distinct_traces(self, service_id: int) -> float:
        return hll_estimate(self.hll[service_id], self.p)


def hll_estimate(regs: np.ndarray, p: int) -> float:
    lib = _lib.load()
    r = np.ascontiguousarray(regs, dtype=np.uint8)
    return float(lib.sa_hll_estimate(r.ctypes.data_as(_lib.u8p), p))


def bucket_thresholds(bounds, unit: str = "ms"):
    lib = _lib.load()
    b = np.ascontiguousarray(bounds, dtype=np.float64)
    thr = np.zeros(max(1, len(b)), dtype=np.uint64)
    nneg = C.c_uint32(0)
    rc = lib.sa_bucket_thresholds(b.ctypes.data_as(_lib.f64p), len(b),
                                  _lib.SA_UNIT_S if unit == "s" else _lib.SA_UNIT_MS,
                                  thr.ctypes.data_as(_lib.u64p), C.byref(nneg))
    if rc != 0:
        raise SpanAggError(rc, "invalid histogram bounds")
    return thr[: len(b) - nneg.value], nneg.value


class _ResultOwner:
    """Frees an sa_red_result once the last numpy view of its columns is gone."""

    def __init__(self, lib, out):
        self.lib, self.out = lib, out

    def __del__(self):
        self.lib.sa_red_result_free(self.out)


def _red_result(owner, rc: int, out, allow_drops: bool, what: str, _fn=None) -> RedResult:
    """numpy views of an sa_red_result's columns (no copy: a C4-scale flush is
    ~170 MB); the result is freed when the last view is collected."""
    lib = owner.lib
    if rc not in (0, _lib.SA_EFULL) or not out:
        owner._check(rc if rc else _lib.SA_ESTATE, what)
    keep = _ResultOwner(lib, out)
    r = out.contents
    n, nb = int(r.n_series), int(r.n_buckets)

    def arr(p, shape, dt):
        if n == 0:
            return np.zeros(shape, dtype=dt)
        count = int(np.prod(shape))
        buf = (C.c_uint64 * count).from_address(C.cast(p, C.c_void_p).value)
        buf._keep = keep  # the views' base holds the result
        return np.frombuffer(buf, dtype=dt).reshape(shape)

    res = RedResult(arr(r.key_hash, (n,), np.uint64), arr(r.bucket_counts, (n, nb), np.uint64),
                    arr(r.calls, (n,), np.uint64), arr(r.sum_ns, (n,), np.uint64),
                    arr(r.sum, (n,), np.float64), rc)
    del keep
    if rc == _lib.SA_EFULL and not allow_drops:
        raise SpanAggError(rc, f"{what}: spans dropped (key table full); stats={owner.stats()}")
    return res


def _sketch_result(lib, out) -> SketchResult:
    try:
        r = out.contents
        hll = np.ctypeslib.as_array(r.hll, shape=(r.n_services, 1 << r.hll_p)).copy()
        cms = np.ctypeslib.as_array(r.cms, shape=(r.cms_d, r.cms_w)).copy()
        return SketchResult(int(r.window_id), hll, cms, int(r.hll_p))
    finally:
        lib.sa_sketch_result_free(out)


def _ptr(x) -> int:
    """Device pointer of a torch tensor, or an int passthrough."""
    if isinstance(x, int):
        return x
    return int(x.data_ptr())


def _expo_result(obj, rc, out, allow_drops, what) -> ExpoResult:
    """sa_exp_result -> ExpoResult (copies), freeing the library's result."""
    if rc not in (0, _lib.SA_EFULL) or not out:
        obj._check(rc if rc else _lib.SA_ESTATE, what)
    try:
        r = out.contents
        n, M = int(r.n_series), int(r.max_size)

        def arr(p, dt):
            return np.zeros(0, dtype=dt) if n == 0 else np.ctypeslib.as_array(p, shape=(n,)).copy()

        bk = np.zeros((0, M), np.uint64) if n == 0 else np.ctypeslib.as_array(r.bucket_counts, shape=(n, M))
        nb = arr(r.n_buckets, np.uint32)
        res = ExpoResult(arr(r.key_hash, np.uint64), arr(r.count, np.uint64), arr(r.zero_count, np.uint64),
                         arr(r.sum_ns, np.uint64), arr(r.sum, np.float64), arr(r.min, np.float64),
                         arr(r.max, np.float64), arr(r.scale, np.int32), arr(r.offset, np.int32),
                         [bk[i, : int(nb[i])].copy() for i in range(n)], rc)
    finally:
        obj.lib.sa_exp_result_free(out)
    if rc == _lib.SA_EFULL and not allow_drops:
        raise SpanAggError(rc, f"{what}: spans dropped (key table full); stats={obj.stats()}")
    return res


class Engine:
    def __init__(self, config: Optional[Config] = None, **kw):
        self.lib = _lib.load()
        self.config = config or Config(**kw)
        c, self._bounds_keepalive = self.config.to_c()
        h = C.c_void_p()
        rc = self.lib.sa_create(C.byref(c), C.byref(h))
        if rc != 0:
            raise SpanAggError(rc, "sa_create failed (is a gfx950 GPU visible?)")
        self._h = h
        self.n_buckets = len(self.config.bounds) + 1

    # -- lifecycle ---------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None):
            self.lib.sa_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int, what: str):
        if rc != 0:
            raise SpanAggError(rc, f"{what}: {self.lib.sa_last_error(self._h).decode()}")

    # -- hot path ----------------------------------------------------------
    def ingest(self, batch: SpanBatch):
        b = _lib.sa_span_batch(*[c.ctypes.data for c in batch.columns()], len(batch))
        self._check(self.lib.sa_ingest(self._h, C.byref(b)), "sa_ingest")

    def ingest_async(self, batch: SpanBatch):
        """sa_ingest_async: columns in sa_host_alloc memory stay the engine's
        until the next ingest_async (or sync) returns."""
        b = _lib.sa_span_batch(*[c.ctypes.data for c in batch.columns()], len(batch))
        self._check(self.lib.sa_ingest_async(self._h, C.byref(b)), "sa_ingest_async")

    def ingest_device(self, key, start, end, w0, w1, meta, n: Optional[int] = None,
                      stream: Optional[int] = None):
        """Device-resident batch: torch tensors (or raw device pointers)."""
        if n is None:
            n = int(key.numel())
        b = _lib.sa_span_batch(_ptr(key), _ptr(start), _ptr(end), _ptr(w0), _ptr(w1),
                               _ptr(meta), n)
        self._check(self.lib.sa_ingest_device(self._h, C.byref(b), C.c_void_p(stream or 0)),
                    "sa_ingest_device")

    def ingest_device_many(self, batches, stream: Optional[int] = None):
        """sa_ingest_device_many: device-resident batches in order, each a
        (key, start, end, w0, w1, meta[, n]) tuple of torch tensors or raw
        device pointers; one HIP graph of launches on small-table engines."""
        arr = (_lib.sa_span_batch * max(1, len(batches)))()
        for i, bt in enumerate(batches):
            cols = bt[:6]
            n = int(bt[6]) if len(bt) > 6 else int(cols[0].numel())
            arr[i] = _lib.sa_span_batch(*[_ptr(c) for c in cols], n)
        self._check(self.lib.sa_ingest_device_many(self._h, arr, len(batches), C.c_void_p(stream or 0)),
                    "sa_ingest_device_many")

    def join(self, stream: Optional[int] = None):
        """sa_join: order `stream` (a hipStream_t handle, None = the engine's)
        after every launch enqueued so far, the binned path's aggregates on
        the engine's own stream included (before timing events on `stream`)."""
        self._check(self.lib.sa_join(self._h, C.c_void_p(stream or 0)), "sa_join")

    def sync(self):
        self._check(self.lib.sa_sync(self._h), "sa_sync")

    # -- export ------------------------------------------------------------
    def flush(self, allow_drops: bool = False) -> RedResult:
        out = C.POINTER(_lib.sa_red_result)()
        rc = self.lib.sa_flush(self._h, C.byref(out))
        return _red_result(self, rc, out, allow_drops, "sa_flush", self.lib.sa_flush)

    def window_read(self, window_id: int) -> SketchResult:
        out = C.POINTER(_lib.sa_sketch_result)()
        self._check(self.lib.sa_window_read(self._h, window_id, C.byref(out)), "sa_window_read")
        return _sketch_result(self.lib, out)

    def flush_exp(self, allow_drops: bool = False) -> ExpoResult:
        out = C.POINTER(_lib.sa_exp_result)()
        rc = self.lib.sa_flush_exp(self._h, C.byref(out))
        return _expo_result(self, rc, out, allow_drops, "sa_flush_exp")

    def reclaim_keys(self, force: bool = False):
        """sa_reclaim_keys: empty the key table (force) or do the flush-time
        policy (more than half full); only right after a flush."""
        self._check(self.lib.sa_reclaim_keys(self._h, int(force)), "sa_reclaim_keys")

    def key_union_probe(self, ids) -> np.ndarray:
        """Diagnostic: the group flush's device key union (sa_key_union_probe)
        of `ids` -- their distinct non-zero values, ascending."""
        a = np.ascontiguousarray(ids, dtype=np.uint64)
        out = np.empty(max(1, len(a)), dtype=np.uint64)
        n = C.c_uint64(0)
        self._check(self.lib.sa_key_union_probe(self._h, a.ctypes.data_as(_lib.u64p), len(a),
                                                out.ctypes.data_as(_lib.u64p), C.byref(n)), "sa_key_union_probe")
        return out[: n.value].copy()

    def expo_probe(self, values, scales):
        """GPU bucket index and Go math.Log of each value (diagnostic)."""
        v = np.ascontiguousarray(values, dtype=np.float64)
        s = np.ascontiguousarray(scales, dtype=np.int32)
        idx = np.zeros(len(v), dtype=np.int32)
        logs = np.zeros(len(v), dtype=np.float64)
        self._check(self.lib.sa_expo_probe(self._h, v.ctypes.data_as(_lib.f64p), s.ctypes.data_as(C.POINTER(C.c_int32)),
                                           len(v), idx.ctypes.data_as(C.POINTER(C.c_int32)),
                                           logs.ctypes.data_as(_lib.f64p)), "sa_expo_probe")
        return idx, logs

    def expo_fast_probe(self, d_ns, scales, log2_err=True):
        """The counting kernel's bucket-index fast path (diagnostic): (fast,
        exact, max log2 error) -- fast[i] is INT32_MIN where it defers to the
        exact path; the error is the hardware log2's over every float in [1, 2)."""
        d = np.ascontiguousarray(d_ns, dtype=np.uint64)
        s = np.ascontiguousarray(scales, dtype=np.int32)
        fast = np.zeros(len(d), dtype=np.int32)
        exact = np.zeros(len(d), dtype=np.int32)
        err = C.c_double(0.0)
        self._check(self.lib.sa_expo_fast_probe(self._h, d.ctypes.data_as(_lib.u64p),
                                                s.ctypes.data_as(C.POINTER(C.c_int32)), len(d),
                                                fast.ctypes.data_as(C.POINTER(C.c_int32)),
                                                exact.ctypes.data_as(C.POINTER(C.c_int32)),
                                                C.byref(err) if log2_err else None), "sa_expo_fast_probe")
        return fast, exact, err.value

    def window_advance(self, new_base: int):
        self._check(self.lib.sa_window_advance(self._h, int(new_base)), "sa_window_advance")

    def stats(self) -> dict:
        s = _lib.sa_stats()
        self._check(self.lib.sa_get_stats(self._h, C.byref(s)), "sa_get_stats")
        return {name: int(getattr(s, name)) for name, _ in _lib.sa_stats._fields_ if name != "pad"}

    # -- multi-GPU merge hooks (device pointers) ----------------------------
    def export_keys(self, d_keys, cap: int, stream: Optional[int] = None) -> int:
        n = C.c_uint64(0)
        self._check(self.lib.sa_export_keys(self._h, C.c_void_p(_ptr(d_keys) if cap else 0), cap,
                                            C.byref(n), C.c_void_p(stream or 0)), "sa_export_keys")
        return int(n.value)

    def gather_dense(self, d_keys, n: int, d_rows, reset: bool, stream: Optional[int] = None):
        self._check(self.lib.sa_gather_dense(self._h, C.c_void_p(_ptr(d_keys) if n else 0), n,
                                             C.c_void_p(_ptr(d_rows) if n else 0), int(reset),
                                             C.c_void_p(stream or 0)), "sa_gather_dense")

    def window_export(self, window_id: int, d_hll, d_cms, stream: Optional[int] = None):
        self._check(self.lib.sa_window_export(self._h, window_id, C.c_void_p(_ptr(d_hll)),
                                              C.c_void_p(_ptr(d_cms)), C.c_void_p(stream or 0)),
                    "sa_window_export")


class Group:
    """One engine per GPU behind one handle (include/spanagg.h sa_group_*):
    host batches shard by trace id (trace_w1 % n), flush and window reads
    return the merge (RCCL over distinct devices, device copies otherwise)."""

    def __init__(self, devices: Sequence[int], config: Optional[Config] = None, **kw):
        self.lib = _lib.load()
        self.config = config or Config(**kw)
        c, self._bounds_keepalive = self.config.to_c()
        devs = (C.c_int32 * len(devices))(*[int(d) for d in devices])
        h = C.c_void_p()
        rc = self.lib.sa_group_create(C.byref(c), devs, len(devices), C.byref(h))
        if rc != 0:
            raise SpanAggError(rc, "sa_group_create failed (are the gfx950 GPUs visible?)")
        self._h = h
        self.n_buckets = len(self.config.bounds) + 1

    def close(self):
        if getattr(self, "_h", None):
            self.lib.sa_group_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int, what: str):
        if rc != 0:
            raise SpanAggError(rc, f"{what}: {self.lib.sa_group_last_error(self._h).decode()}")

    @property
    def size(self) -> int:
        return int(self.lib.sa_group_size(self._h))

    @property
    def uses_rccl(self) -> bool:
        return bool(self.lib.sa_group_uses_rccl(self._h))

    def ingest(self, batch: SpanBatch):
        b = _lib.sa_span_batch(*[c.ctypes.data for c in batch.columns()], len(batch))
        self._check(self.lib.sa_group_ingest(self._h, C.byref(b)), "sa_group_ingest")

    def ingest_device(self, key, start, end, w0, w1, meta, n: Optional[int] = None, src: int = 0,
                      stream: Optional[int] = None):
        """sa_group_ingest_device: a batch in HBM of member `src`'s device
        (torch tensors or raw device pointers), partitioned by trace id on
        that device and ingested by every member on its own stream."""
        if n is None:
            n = int(key.numel())
        b = _lib.sa_span_batch(_ptr(key), _ptr(start), _ptr(end), _ptr(w0), _ptr(w1), _ptr(meta), n)
        self._check(self.lib.sa_group_ingest_device(self._h, C.byref(b), int(src), C.c_void_p(stream or 0)),
                    "sa_group_ingest_device")

    def sync(self):
        self._check(self.lib.sa_group_sync(self._h), "sa_group_sync")

    def flush(self, allow_drops: bool = False) -> RedResult:
        out = C.POINTER(_lib.sa_red_result)()
        rc = self.lib.sa_group_flush(self._h, C.byref(out))
        return _red_result(self, rc, out, allow_drops, "sa_group_flush")

    def flush_exp(self, allow_drops: bool = False) -> ExpoResult:
        """sa_group_flush_exp: the members' exponential histograms, folded."""
        out = C.POINTER(_lib.sa_exp_result)()
        rc = self.lib.sa_group_flush_exp(self._h, C.byref(out))
        return _expo_result(self, rc, out, allow_drops, "sa_group_flush_exp")

    def window_read(self, window_id: int) -> SketchResult:
        out = C.POINTER(_lib.sa_sketch_result)()
        self._check(self.lib.sa_group_window_read(self._h, window_id, C.byref(out)), "sa_group_window_read")
        return _sketch_result(self.lib, out)

    def window_advance(self, new_base: int):
        self._check(self.lib.sa_group_window_advance(self._h, int(new_base)), "sa_group_window_advance")

    def stats(self) -> dict:
        s = _lib.sa_stats()
        self._check(self.lib.sa_group_get_stats(self._h, C.byref(s)), "sa_group_get_stats")
        return {name: int(getattr(s, name)) for name, _ in _lib.sa_stats._fields_ if name != "pad"}
