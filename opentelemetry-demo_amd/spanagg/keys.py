"""Dimension-key building and hashing on the host (the device only sees u64 ids).

Restates the connector's key identity ([UPSTREAM] spanmetricsconnector
connector.go `buildKey` + `concatDimensionValue`):

    key = service.name \\0 span.name \\0 SpanKindStr \\0 StatusCodeStr [\\0 dim]*

Parts listed in exclude_dimensions are omitted; a configured dimension that is
absent on both span and resource (and has no default) is skipped with no
separator; non-string values are keyed by their AsString() form.  Series are
grouped by resource first (A10), so the device-side series id is
xxh64(resource_hash LE || key bytes).  The hash function is xxHash64 (the Go
module uses cespare/xxhash/v2); this host uses the `xxhash` package for it.
"""
from __future__ import annotations

import json
from typing import Iterable, Mapping, Optional, Sequence

import xxhash

SPAN_KIND_STR = ("SPAN_KIND_UNSPECIFIED", "SPAN_KIND_INTERNAL", "SPAN_KIND_SERVER",
                 "SPAN_KIND_CLIENT", "SPAN_KIND_PRODUCER", "SPAN_KIND_CONSUMER")
STATUS_CODE_STR = ("STATUS_CODE_UNSET", "STATUS_CODE_OK", "STATUS_CODE_ERROR")

SERVICE_NAME_KEY = "service.name"
SPAN_NAME_KEY = "span.name"
SPAN_KIND_KEY = "span.kind"
STATUS_CODE_KEY = "status.code"


def span_kind_str(kind: int) -> str:
    """traceutil.SpanKindStr: out-of-range -> "" (A7)."""
    return SPAN_KIND_STR[kind] if 0 <= kind < len(SPAN_KIND_STR) else ""


def status_code_str(code: int) -> str:
    """traceutil.StatusCodeStr: out-of-range -> "" (A7)."""
    return STATUS_CODE_STR[code] if 0 <= code < len(STATUS_CODE_STR) else ""


def as_string(v) -> str:
    """pcommon.Value.AsString() for the value kinds the host meets."""
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, int):
        return str(v)
    if isinstance(v, float):
        if v != v:
            return "NaN"
        if v in (float("inf"), float("-inf")):
            return "+Inf" if v > 0 else "-Inf"
        # Go strconv.FormatFloat(f, 'f', -1, 64): shortest round-trip digits,
        # positional notation, no trailing ".0"
        import numpy as np
        return np.format_float_positional(v, unique=True, trim="-")
    if isinstance(v, (bytes, bytearray)):
        import base64
        return base64.b64encode(bytes(v)).decode()
    if isinstance(v, (list, tuple, dict)):
        return json.dumps(v, separators=(",", ":"))
    if v is None:
        return ""
    return str(v)


def build_key(service: str, span_name: str, kind: int, status: int,
              dims: Sequence[tuple] = (), span_attrs: Optional[Mapping] = None,
              resource_attrs: Optional[Mapping] = None,
              exclude: Iterable[str] = ()) -> bytes:
    """buildKey: NUL-joined; `dims` is a list of (name, default_or_None)."""
    ex = set(exclude)
    parts: list[str] = []
    if SERVICE_NAME_KEY not in ex:
        parts.append(service)
    if SPAN_NAME_KEY not in ex:
        parts.append(span_name)
    if SPAN_KIND_KEY not in ex:
        parts.append(span_kind_str(kind))
    if STATUS_CODE_KEY not in ex:
        parts.append(status_code_str(status))
    span_attrs = span_attrs or {}
    resource_attrs = resource_attrs or {}
    out = "\x00".join(parts)
    for name, default in dims:
        if name in span_attrs:
            v = span_attrs[name]
        elif name in resource_attrs:
            v = resource_attrs[name]
        elif default is not None:
            v = default
        else:
            continue  # A5: missing optional dimension, no separator
        out += "\x00" + as_string(v)
    return out.encode("utf-8")


def resource_hash(attrs: Mapping) -> int:
    """Resource identity (stand-in for pdatautil.MapHash): xxh64 over the
    attributes in key order, each as key \\0 AsString(value) \\0 type tag."""
    h = xxhash.xxh64(seed=0)
    for k in sorted(attrs):
        v = attrs[k]
        h.update(k.encode())
        h.update(b"\x00")
        h.update(as_string(v).encode())
        h.update(b"\x00" + type(v).__name__.encode() + b"\x01")
    return h.intdigest()


def series_hash_seeded(res_hash: int, key: bytes, seed: int) -> int:
    return xxhash.xxh64_intdigest(res_hash.to_bytes(8, "little") + key, seed=seed)


def assign_series_id(res_hash: int, key: bytes, owner) -> tuple:
    """Series id of (resource, key): xxh64 with seed 0, 1, ... until the id is
    neither 0 (reserved by the engine) nor held by another series (owner(id)
    -> None free, True this series, False another).  Returns (id, seed)."""
    seed = 0
    while True:
        h = series_hash_seeded(res_hash, key, seed)
        if h != 0 and owner(h) is not False:
            return h, seed
        seed += 1


def series_hash(res_hash: int, key: bytes) -> int:
    """Device series id with nothing else interned (seed 0; seed 1 if that is 0)."""
    return assign_series_id(res_hash, key, lambda h: None)[0]


class KeyDictionary:
    """Host dictionary series id -> (resource attrs, key bytes, datapoint attrs).
    A 64-bit collision (a distinct (resource, key) on a taken id) is re-salted."""

    def __init__(self):
        self._by_id: dict[int, tuple] = {}
        self.collisions = 0

    def intern(self, res_hash: int, key: bytes, resource_attrs: Mapping, dp_attrs: Mapping) -> int:
        """A distinct (resource, key) whose id is taken is re-salted (counted)."""
        def owner(h):
            cur = self._by_id.get(h)
            return None if cur is None else (cur[0] == res_hash and cur[1] == key)

        sid, seed = assign_series_id(res_hash, key, owner)
        if sid not in self._by_id:
            self.collisions += seed > 0
            # attributes are taken from the first span seen for the key (A5/A6)
            self._by_id[sid] = (res_hash, key, dict(resource_attrs), dict(dp_attrs))
        return sid

    def __getitem__(self, sid: int):
        return self._by_id[sid]

    def __contains__(self, sid: int) -> bool:
        return sid in self._by_id

    def __len__(self):
        return len(self._by_id)
