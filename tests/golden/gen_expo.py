#!/usr/bin/env python3
"""Generates tests/golden/expo_kat.json -- TEST INFRASTRUCTURE.

Known answers for the spanmetrics connector's exponential histogram
(`histogram.exponential.max_size`, [UPSTREAM] spanmetricsconnector v0.125.0
internal/metrics `exponentialHistogram.Observe` -> github.com/lightstep/
go-expohisto structure.Histogram[float64].Update), restated in pure Python:

- go_log: Go's math.Log (src/math/log.go: Frexp reduction, the fdlibm
  polynomial, k*Ln2Hi - ((hfsq - (s*(hfsq+R) + k*Ln2Lo)) - f)); CPython
  floats are IEEE doubles with no contraction, so the bits are Go's.
- map_to_index: go-expohisto's mappings -- logarithm (scale 1..20: exact
  powers of two -> (exp << scale) - 1, else floor(Log(v) * Ldexp(Log2E,
  scale))) and exponent (scale <= 0: (base2 exponent + correction) >> -scale).
- Histogram: Update as go-expohisto does it, one value at a time: start at
  scale 20; a value whose index would widen the positive range to maxSize or
  more downscales by the least shift that fits (changeScale), merging
  buckets pairwise; zeros go to zero_count; sum is float64 in arrival order.

The Go module is not in the container and Go is absent: these vectors pin the
C oracle and the GPU kernel to this restatement (parity vs Go itself is
unpinned).  Run: python tests/golden/gen_expo.py
"""
from __future__ import annotations

import json
import math
import os
import random
import struct

LN2HI = 6.93147180369123816490e-01
LN2LO = 1.90821492927058770002e-10
L1, L2, L3, L4 = 6.666666666666735130e-01, 3.999999999940941908e-01, 2.857142874366239149e-01, 2.222219843214978396e-01
L5, L6, L7 = 1.818357216161805012e-01, 1.531383769920937332e-01, 1.479819860511658591e-01
SQRT2_2 = 1.4142135623730951 / 2
LOG2E = 1.4426950408889634  # math.Log2E as float64
MAX_SCALE, MIN_SCALE = 20, -10


def go_log(x: float) -> float:
    assert x > 0 and math.isfinite(x)
    f1, ki = math.frexp(x)
    if f1 < SQRT2_2:
        f1 *= 2
        ki -= 1
    f = f1 - 1
    k = float(ki)
    s = f / (2 + f)
    s2 = s * s
    s4 = s2 * s2
    t1 = s2 * (L1 + s4 * (L3 + s4 * (L5 + s4 * L7)))
    t2 = s4 * (L2 + s4 * (L4 + s4 * L6))
    R = t1 + t2
    hfsq = 0.5 * f * f
    return k * LN2HI - ((hfsq - (s * (hfsq + R) + k * LN2LO)) - f)


def bits(x: float) -> int:
    return struct.unpack("<Q", struct.pack("<d", x))[0]


def map_to_index(v: float, scale: int) -> int:
    b = bits(v)
    raw_exp = (b >> 52) & 0x7FF
    sig = b & ((1 << 52) - 1)
    if scale > 0:
        if v <= 2.0 ** -1022:
            return -1022 << scale
        if sig == 0:
            return ((raw_exp - 1023) << scale) - 1
        idx = math.floor(go_log(v) * math.ldexp(LOG2E, scale))
        return min(idx, ((1023 + 1) << scale) - 1)
    if raw_exp == 0:  # subnormal
        raw_exp -= (64 - sig.bit_length()) - 12
    exp = raw_exp - 1023
    correction = -1 if sig == 0 else 0
    return (exp + correction) >> (-scale)


class Histogram:
    """go-expohisto structure.Histogram[float64] for non-negative values."""

    def __init__(self, max_size: int):
        self.max_size = max_size
        self.scale = MAX_SCALE
        self.count = 0
        self.zero = 0
        self.sum = 0.0
        self.min = self.max = 0.0
        self.start = self.end = None  # positive index range
        self.counts: dict[int, int] = {}

    def _change_scale(self, high: int, low: int) -> int:
        change = 0
        while high - low >= self.max_size:
            high >>= 1
            low >>= 1
            change += 1
        return change

    def _downscale(self, change: int):
        if change <= 0:
            return
        merged: dict[int, int] = {}
        for i, c in self.counts.items():
            merged[i >> change] = merged.get(i >> change, 0) + c
        self.counts = merged
        self.start >>= change
        self.end >>= change
        self.scale -= change

    def _increment(self, index: int):
        if self.start is None:
            self.start = self.end = index
        elif index < self.start:
            if self.end - index >= self.max_size:
                return (self.end, index)
            self.start = index
        elif index > self.end:
            if index - self.start >= self.max_size:
                return (index, self.start)
            self.end = index
        self.counts[index] = self.counts.get(index, 0) + 1
        return None

    def update(self, v: float):
        if self.count == 0:
            self.min = self.max = v
        else:
            self.min = min(self.min, v)
            self.max = max(self.max, v)
        self.count += 1
        if v == 0:
            self.zero += 1
            return
        self.sum += v
        hl = self._increment(map_to_index(v, self.scale))
        if hl is not None:
            self._downscale(self._change_scale(*hl))
            assert self._increment(map_to_index(v, self.scale)) is None

    def result(self):
        out = dict(count=self.count, zero_count=self.zero, sum=self.sum.hex(), min=float(self.min).hex(),
                   max=float(self.max).hex(), scale=self.scale if self.start is not None else MAX_SCALE,
                   offset=0, counts=[])
        if self.start is not None:
            out["offset"] = self.start
            out["counts"] = [self.counts.get(i, 0) for i in range(self.start, self.end + 1)]
        return out


def durations(rng, n):
    """ns durations: lognormal around 5 ms plus the edges: zeros, exact
    powers of two in ms, +-1 ns around them, sub-microsecond and very long."""
    ds = [int(math.exp(rng.gauss(math.log(5e6), 1.5))) for _ in range(n)]
    edge = [0, 0, 1, 2, 3, 999, 1000, 1_000_000, 1_000_001, 999_999, 500_000, 250_000, 2_000_000, 4_000_000,
            1 << 20, 60_000_000_000, 3_600_000_000_000]
    for k in range(-6, 16):
        t = int(round((2.0 ** k) * 1e6))
        edge += [t - 1, t, t + 1]
    ds += edge
    rng.shuffle(ds)
    return ds


def case(name, ds, max_size, unit):
    div = 1e9 if unit == "s" else 1e6
    h = Histogram(max_size)
    for d in ds:
        h.update(float(d) / div)
    return dict(name=name, unit=unit, max_size=max_size, durations_ns=ds, expected=h.result())


def main():
    rng = random.Random(20261016)
    cases = [
        case("lognormal_default_size", durations(rng, 3000), 160, "ms"),
        case("lognormal_small_size", durations(rng, 2000), 8, "ms"),
        case("narrow_range_high_scale", [5_000_000 + rng.randrange(1000) for _ in range(500)], 160, "ms"),
        case("one_value", [7_340_032], 160, "ms"),
        case("zeros_only", [0, 0, 0], 160, "ms"),
        case("seconds_unit", durations(rng, 1000), 40, "s"),
        case("size_two", durations(rng, 300), 2, "ms"),
    ]
    logs = []
    for x in [1e-6, 1e-3, 0.5, 0.7071067811865476, 0.7071067811865475, 1.0, 1.0000000001, 2.0, 3.0, 5.0,
              7.340032, 1e3, 6e4, 3.6e6, 1e300, 2.0 ** -1000] + [rng.uniform(1e-3, 1e5) for _ in range(200)]:
        logs.append([float(x).hex(), go_log(float(x)).hex()])
    idx = []
    for d in durations(rng, 300):
        if d == 0:
            continue
        v = float(d) / 1e6
        for s in (20, 13, 5, 1, 0, -2):
            idx.append([d, s, map_to_index(v, s)])
    out = dict(note="generated by tests/golden/gen_expo.py (pure-Python restatement; see its header)",
               cases=cases, go_log=logs, map_to_index_ms=idx)
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "expo_kat.json")
    with open(path, "w") as f:
        json.dump(out, f, separators=(",", ":"))
        f.write("\n")
    print(path, len(cases), "cases")


if __name__ == "__main__":
    main()
