"""spanagg -- host side of the MI355X span-aggregation engine.

The hot path (per-span RED aggregation + HLL / count-min sketches) runs in
libspanagg.so's HIP kernels; this package binds its C-ABI, builds and hashes
dimension keys, generates synthetic workloads and merges partials across
ranks.  Importing it does not require a GPU; creating an Engine does.
"""
from .engine import (DEFAULT_BOUNDS_MS, Config, Engine, Group, RedResult, SketchResult, SpanBatch,
                     bucket_thresholds, hll_estimate, pack_meta, trace_words)
from ._lib import SpanAggError, load

__all__ = [
    "DEFAULT_BOUNDS_MS", "Config", "Engine", "Group", "RedResult", "SketchResult", "SpanBatch",
    "SpanAggError", "bucket_thresholds", "hll_estimate", "load", "pack_meta", "trace_words",
]
