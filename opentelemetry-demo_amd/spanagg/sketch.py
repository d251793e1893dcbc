"""Host-side queries over one window's sketches (SURVEY.md rows a16-a17 and
Appendix C): count-min point queries, heavy hitters over the known ERROR
series, HLL estimates per service, and a simple per-window anomaly flag."""
from __future__ import annotations

from typing import Iterable, Sequence

import numpy as np

from .engine import hll_estimate

CMS_SEEDS = (0x9E3779B97F4A7C15, 0xBF58476D1CE4E5B9, 0x94D049BB133111EB, 0xD6E8FEB86659FD93,
             0xA0761D6478BD642F, 0xE7037ED1A0B428DB, 0x8EBC6AF09C88C6E3, 0x589965CC75374CC3)
M64 = (1 << 64) - 1


def _splitmix64(x: int) -> int:
    z = (x + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def cms_query(cms: np.ndarray, key_hash: int) -> int:
    """min_j cms[j][splitmix64(key ^ seed_j) >> (64 - log2 w)]: an upper bound on
    the key's ERROR spans in the window (exact when no collision)."""
    d, w = cms.shape
    shift = 64 - (w.bit_length() - 1)
    return int(min(cms[j, _splitmix64(int(key_hash) ^ CMS_SEEDS[j]) >> shift] for j in range(d)))


def heavy_hitters(cms: np.ndarray, error_keys: Iterable[int], k: int = 10):
    """Top-k (key, estimate) over the host's ERROR series (status code 2 keys)."""
    est = [(int(key), cms_query(cms, key)) for key in error_keys]
    est = [e for e in est if e[1] > 0]
    est.sort(key=lambda e: (-e[1], e[0]))
    return est[:k]


def distinct_traces(hll: np.ndarray, p: int) -> np.ndarray:
    """[n_services] HLL estimates of distinct trace ids."""
    return np.array([hll_estimate(hll[s], p) for s in range(hll.shape[0])])


def anomalous(series: Sequence[float], factor: float, min_base: float = 1.0) -> list:
    """Indices whose value exceeds `factor` x the series median (floor min_base)."""
    x = np.asarray(series, dtype=np.float64)
    base = max(float(np.median(x)), min_base)
    return [i for i, v in enumerate(x) if v > factor * base]
