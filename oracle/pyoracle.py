"""ctypes wrapper of the CPU oracle (oracle/build/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg as the checker / CPU baseline, never by the
product package.  Build with `make -C oracle`.
"""
from __future__ import annotations

import ctypes as C
import os
import time

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")

DEFAULT_BOUNDS_MS = (2, 4, 6, 8, 10, 50, 100, 200, 400, 800, 1000, 1400, 2000, 5000, 10000, 15000)

_u64p = C.POINTER(C.c_uint64)
_u32p = C.POINTER(C.c_uint32)
_u8p = C.POINTER(C.c_uint8)
_f64p = C.POINTER(C.c_double)
_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"oracle not built: {LIB_PATH} (run `make -C oracle`)")
        L = C.CDLL(LIB_PATH)
        L.or_xxh64.restype = C.c_uint64
        L.or_xxh64.argtypes = [C.c_void_p, C.c_size_t, C.c_uint64]
        L.or_search_float64s.restype = C.c_uint32
        L.or_search_float64s.argtypes = [_f64p, C.c_uint32, C.c_double]
        L.or_duration.restype = C.c_double
        L.or_duration.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32]
        L.or_splitmix64.restype = C.c_uint64
        L.or_splitmix64.argtypes = [C.c_uint64]
        L.or_hll_estimate.restype = C.c_double
        L.or_hll_estimate.argtypes = [_u8p, C.c_uint32]
        L.or_create.restype = C.c_void_p
        L.or_create.argtypes = [_f64p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                C.c_uint32, C.c_uint64, C.c_uint32]
        L.or_destroy.argtypes = [C.c_void_p]
        L.or_ingest.argtypes = [C.c_void_p] + [C.c_void_p] * 6 + [C.c_uint64]
        L.or_ingest_red.argtypes = [C.c_void_p] + [C.c_void_p] * 3 + [C.c_uint64]
        L.or_n_series.restype = C.c_uint64
        L.or_n_series.argtypes = [C.c_void_p]
        L.or_series.argtypes = [C.c_void_p] + [C.c_void_p] * 5
        L.or_reset_red.argtypes = [C.c_void_p]
        L.or_n_windows.restype = C.c_uint64
        L.or_n_windows.argtypes = [C.c_void_p]
        L.or_window_ids.argtypes = [C.c_void_p, C.c_void_p]
        L.or_window.restype = C.c_int
        L.or_window.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p]
        L.or_stats.argtypes = [C.c_void_p, C.c_void_p]
        L.or_go_log.restype = C.c_double
        L.or_go_log.argtypes = [C.c_double]
        L.or_expo_index.restype = C.c_int32
        L.or_expo_index.argtypes = [C.c_double, C.c_int32]
        L.or_expo_series.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint32] + [C.c_void_p] * 9
        L.or_aggregate_strings.restype = C.c_uint64
        L.or_aggregate_strings.argtypes = [C.c_void_p] + [C.c_void_p] * 6 + [
            C.c_uint64, _f64p, C.c_uint32, _u64p]
        _lib = L
    return _lib


def xxh64(data: bytes, seed: int = 0) -> int:
    return int(load().or_xxh64(data, len(data), seed))


def search_float64s(bounds, x: float) -> int:
    b = np.ascontiguousarray(bounds, dtype=np.float64)
    return int(load().or_search_float64s(b.ctypes.data_as(_f64p), len(b), float(x)))


def duration(start: int, end: int, unit_seconds: bool = False) -> float:
    return float(load().or_duration(start, end, int(unit_seconds)))


def splitmix64(x: int) -> int:
    return int(load().or_splitmix64(x))


def hll_estimate(regs, p: int) -> float:
    r = np.ascontiguousarray(regs, dtype=np.uint8)
    return float(load().or_hll_estimate(r.ctypes.data_as(_u8p), p))


def go_log(x: float) -> float:
    return float(load().or_go_log(float(x)))


def expo_index(v: float, scale: int) -> int:
    return int(load().or_expo_index(float(v), int(scale)))


def expo_series(start, end, max_size: int = 160, unit_seconds: bool = False) -> dict:
    """One series' exponential histogram, values observed in the given order."""
    st = np.ascontiguousarray(start, dtype=np.uint64)
    en = np.ascontiguousarray(end, dtype=np.uint64)
    cnt, zero = C.c_uint64(), C.c_uint64()
    sm, mn, mx = C.c_double(), C.c_double(), C.c_double()
    sc, off, nb = C.c_int32(), C.c_int32(), C.c_uint32()
    counts = np.zeros(max(1, max_size), dtype=np.uint64)
    load().or_expo_series(st.ctypes.data, en.ctypes.data, len(st), max_size, int(unit_seconds), C.byref(cnt),
                          C.byref(zero), C.byref(sm), C.byref(mn), C.byref(mx), C.byref(sc), C.byref(off),
                          C.byref(nb), counts.ctypes.data)
    return dict(count=cnt.value, zero_count=zero.value, sum=sm.value, min=mn.value, max=mx.value,
                scale=sc.value, offset=off.value, counts=counts[: nb.value].copy())


def expo_aggregate(batch, max_size: int = 160, unit_seconds: bool = False) -> dict:
    """Exponential histograms of every non-zero series of a batch (spans of
    one series in arrival order), keyed by series id."""
    key = np.asarray(batch.key_hash)
    order = np.argsort(key, kind="stable")
    k_sorted = key[order]
    bounds = np.flatnonzero(np.diff(k_sorted)) + 1
    out = {}
    for grp in np.split(order, bounds):
        k = int(key[grp[0]])
        if k == 0:
            continue
        out[k] = expo_series(np.asarray(batch.start_ns)[grp], np.asarray(batch.end_ns)[grp], max_size, unit_seconds)
    return out


class Oracle:
    """Go-faithful spanmetrics aggregation + reference sketches over SoA v1."""

    def __init__(self, bounds=DEFAULT_BOUNDS_MS, unit="ms", hll_p=14, cms_d=4, cms_w=2048,
                 window_ns=10_000_000_000, n_services=64):
        L = load()
        self.bounds = np.ascontiguousarray(bounds, dtype=np.float64)
        self.nbk = len(self.bounds) + 1
        self.n_services, self.hll_p, self.cms_d, self.cms_w = n_services, hll_p, cms_d, cms_w
        b = self.bounds if len(self.bounds) else np.zeros(1)
        self._h = L.or_create(b.ctypes.data_as(_f64p), len(self.bounds), int(unit == "s"), hll_p,
                              cms_d, cms_w, window_ns, n_services)
        if not self._h:
            raise ValueError("bad oracle config")

    def close(self):
        if self._h:
            load().or_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def ingest(self, batch):
        cols = [np.ascontiguousarray(c) for c in batch.columns()]
        load().or_ingest(self._h, *[c.ctypes.data for c in cols], len(cols[0]))

    def ingest_red(self, batch):
        cols = [np.ascontiguousarray(c) for c in batch.columns()[:3]]
        load().or_ingest_red(self._h, *[c.ctypes.data for c in cols], len(cols[0]))

    def series(self):
        n = int(load().or_n_series(self._h))
        key = np.zeros(n, np.uint64)
        counts = np.zeros((n, self.nbk), np.uint64)
        sum_go = np.zeros(n, np.float64)
        sum_ns = np.zeros(n, np.uint64)
        calls = np.zeros(n, np.uint64)
        if n:
            load().or_series(self._h, key.ctypes.data, counts.ctypes.data, sum_go.ctypes.data,
                             sum_ns.ctypes.data, calls.ctypes.data)
        return dict(key_hash=key, bucket_counts=counts, sum_go=sum_go, sum_ns=sum_ns, calls=calls)

    def reset_red(self):
        load().or_reset_red(self._h)

    def window_ids(self):
        n = int(load().or_n_windows(self._h))
        ids = np.zeros(n, np.uint64)
        if n:
            load().or_window_ids(self._h, ids.ctypes.data)
        return [int(x) for x in ids]

    def window(self, wid: int):
        hll = np.zeros((self.n_services, 1 << self.hll_p), np.uint8)
        cms = np.zeros((self.cms_d, self.cms_w), np.uint32)
        if load().or_window(self._h, wid, hll.ctypes.data, cms.ctypes.data) != 0:
            raise KeyError(wid)
        return hll, cms

    def stats(self):
        s = np.zeros(3, np.uint64)
        load().or_stats(self._h, s.ctypes.data)
        return dict(spans=int(s[0]), invalid_service=int(s[1]), zero_key=int(s[2]))


def aggregate_strings(strings, svc_id, name_id, kind, status, start, end, bounds=DEFAULT_BOUNDS_MS):
    """Reference-faithful string-keyed aggregation (CPU baseline). Returns
    (n_series, checksum, seconds)."""
    L = load()
    enc = [s.encode() for s in strings]
    arr = (C.c_char_p * len(enc))(*enc)
    cols = [np.ascontiguousarray(x, dtype=np.uint32) for x in (svc_id, name_id, kind, status)]
    st = np.ascontiguousarray(start, dtype=np.uint64)
    en = np.ascontiguousarray(end, dtype=np.uint64)
    b = np.ascontiguousarray(bounds, dtype=np.float64)
    cs = C.c_uint64(0)
    t = time.perf_counter()
    n = L.or_aggregate_strings(C.cast(arr, C.c_void_p), *[c.ctypes.data for c in cols],
                               st.ctypes.data, en.ctypes.data, len(st), b.ctypes.data_as(_f64p),
                               len(b), C.byref(cs))
    return int(n), int(cs.value), time.perf_counter() - t
