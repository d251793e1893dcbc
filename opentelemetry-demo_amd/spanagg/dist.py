"""Cross-GPU merge of span-aggregation partials (one process per GPU).

Spans are sharded by trace id across ranks, so the hot path has
no data-path collective; the only exchange is at flush / window close:

  1. every rank exports the series ids it holds a non-zero delta for;
  2. all_gather of those id lists -> the same sorted union on every rank
     (this fixes one dense index, since each GPU's hash-table slots differ);
  3. each rank densifies its counters against the union ([U][n_buckets+1] u64:
     bucket counts + ns sum) and the ranks all_reduce(SUM) them;
  4. HLL registers all_reduce(MAX) (u8; max-merge is exact and idempotent) and
     count-min cells all_reduce(SUM) (u64, saturated to u32 on read).

On MI355X the process group is `nccl` (= RCCL over xGMI); tests run the same
code on `gloo` with CPU tensors.  The local side is any object implementing
`LocalPartial` -- the GPU `EnginePartial` below, or a test adapter.
"""
from __future__ import annotations

from typing import Optional, Protocol, Tuple

import numpy as np
import torch
import torch.distributed as dist

from .engine import Engine, RedResult


class LocalPartial(Protocol):
    n_buckets: int
    device: torch.device

    def export_keys(self) -> torch.Tensor: ...            # int64 [n] series ids (u64 bits)

    def gather_dense(self, keys: torch.Tensor, reset: bool) -> torch.Tensor: ...  # int64 [U, nb+1]

    def window(self, window_id: int) -> Tuple[torch.Tensor, torch.Tensor]: ...  # u8 [S,m], i64 [d,w]


class EnginePartial:
    """LocalPartial over one libspanagg engine (device tensors on its GPU)."""

    def __init__(self, engine: Engine, device: Optional[torch.device] = None):
        self.engine = engine
        self.n_buckets = engine.n_buckets
        self.unit_div = 1e9 if engine.config.unit == "s" else 1e6
        self.device = device or torch.device("cuda", engine.config.device)
        self._cap = 1 << 16

    def _stream(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream

    def export_keys(self) -> torch.Tensor:
        while True:
            buf = torch.empty(self._cap, dtype=torch.int64, device=self.device)
            n = self.engine.export_keys(buf, self._cap, stream=self._stream())
            if n <= self._cap:
                return buf[:n]
            self._cap = 1 << int(n - 1).bit_length()

    def gather_dense(self, keys: torch.Tensor, reset: bool) -> torch.Tensor:
        keys = keys.contiguous()
        rows = torch.empty((keys.numel(), self.n_buckets + 1), dtype=torch.int64, device=self.device)
        self.engine.gather_dense(keys, keys.numel(), rows, reset, stream=self._stream())
        return rows

    def window(self, window_id: int):
        c = self.engine.config
        hll = torch.empty((c.n_services, 1 << c.hll_p), dtype=torch.uint8, device=self.device)
        cms = torch.empty((c.cms_d, c.cms_w), dtype=torch.int64, device=self.device)
        self.engine.window_export(window_id, hll, cms, stream=self._stream())
        return hll, cms


def _all_gather_varlen(t: torch.Tensor, group) -> torch.Tensor:
    world = dist.get_world_size(group)
    n = torch.tensor([t.numel()], dtype=torch.int64, device=t.device)
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n, group=group)
    sizes = [int(x.item()) for x in ns]
    m = max(sizes) if sizes else 0
    if m == 0:
        return t[:0]
    pad = torch.zeros(m, dtype=t.dtype, device=t.device)
    pad[: t.numel()] = t
    outs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(outs, pad, group=group)
    return torch.cat([o[:s] for o, s in zip(outs, sizes)])


def key_union(local_keys: torch.Tensor, group=None) -> torch.Tensor:
    """Sorted union of every rank's series ids (identical on all ranks)."""
    allk = _all_gather_varlen(local_keys, group)
    u = torch.unique(allk)  # sorted (as int64; a fixed order is all that matters)
    return u[u != 0]


def merge_red(local: LocalPartial, group=None, reset: bool = True) -> RedResult:
    """Merged delta RED state across the group (returned on every rank)."""
    union = key_union(local.export_keys(), group)
    rows = local.gather_dense(union, reset)
    if union.numel():
        dist.all_reduce(rows, op=dist.ReduceOp.SUM, group=group)
    keys = union.cpu().numpy().view(np.uint64)
    rows = rows.cpu().numpy().view(np.uint64)
    order = np.argsort(keys, kind="stable")
    keys, rows = keys[order], rows[order]
    nb = local.n_buckets
    counts = np.ascontiguousarray(rows[:, :nb])
    sum_ns = np.ascontiguousarray(rows[:, nb])
    return RedResult(keys, counts, counts.sum(axis=1, dtype=np.uint64), sum_ns,
                     sum_ns.astype(np.float64) / getattr(local, "unit_div", 1e6))


def merge_window(local: LocalPartial, window_id: int, group=None):
    """Merged (hll u8 [S,m], cms u32 [d,w]) of one window across the group."""
    hll, cms = local.window(window_id)
    dist.all_reduce(hll, op=dist.ReduceOp.MAX, group=group)
    dist.all_reduce(cms, op=dist.ReduceOp.SUM, group=group)
    cms_np = cms.cpu().numpy()
    return hll.cpu().numpy(), np.minimum(cms_np, 0xFFFFFFFF).astype(np.uint32)


def shard_of(trace_w1: np.ndarray, world: int) -> np.ndarray:
    """Rank owning each span: trace_id bytes 8..15 (LE word) mod world, so every
    trace's spans land on one GPU."""
    return (np.asarray(trace_w1, dtype=np.uint64) % np.uint64(world)).astype(np.int64)
