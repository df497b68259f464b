"""Multi-GPU sharding of one sampler: one process per GPU.

The sweep reads only the snapshot (GibbsSampling.fs:940-942), so every sequence is
independent given two integer aggregates (count matrix C, background totals T).
Each rank holds a contiguous shard of the sequences, balanced by total length;
once per sweep the ranks sum their partial aggregates with one in-place RCCL
all-reduce (inside libgibbs_hip.so, on its stream).  Uniforms are keyed by the
global sequence index, so results are bit-identical for any number of ranks.
"""
from __future__ import annotations

from typing import Sequence

import numpy as np


def shard_bounds(lengths: Sequence[int], world: int) -> list[tuple[int, int]]:
    """Contiguous [lo, hi) per rank with near-equal sum of lengths (every rank gets
    at least one sequence when there are at least `world` of them)."""
    lengths = np.asarray(lengths, np.int64)
    n = len(lengths)
    if world < 1:
        raise ValueError("world must be >= 1")
    if n == 0:
        return [(0, 0)] * world
    csum = np.concatenate([[0], np.cumsum(lengths)])
    total = csum[-1]
    cuts = [0]
    for r in range(1, world):
        c = int(np.searchsorted(csum, total * r / world, side="left"))
        lo_b = cuts[-1] + 1 if n >= world else cuts[-1]  # at least one sequence per rank
        hi_b = n - (world - r) if n >= world else n
        cuts.append(min(max(c, lo_b), hi_b))
    cuts.append(n)
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def exchange_unique_id(rank: int, group=None) -> bytes:
    """Rank 0 creates the RCCL unique id; every rank receives it via torch.distributed
    (any backend, e.g. gloo)."""
    import torch.distributed as dist

    from ._native import Context
    obj = [Context.unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0, group=group)
    return obj[0]


def open_exchange(ctx, rank: int, world: int, group=None) -> str:
    """The in-kernel aggregate exchange (include/gibbs_hip.h gs_exchange_*): every
    rank's exchange-buffer IPC handle all-gathered over torch.distributed (any backend),
    then opened; the ranks agree before any sweeps (an all-reduce of the outcome, which
    is also the barrier: no rank sweeps before every buffer is open).  From then on the
    live and long sweeps sum the ranks' partial aggregates in their last workgroup (no
    all-reduce after them); the snapshot's first aggregates still go through the
    communicator (gs_state_set_positions).  Returns "" when every rank opened it, else
    the reason (every rank then has it closed: the communicator's all-reduce stays)."""
    import torch
    import torch.distributed as dist
    err = ""
    try:
        h = ctx.exchange_handle()
    except Exception as e:  # noqa: BLE001 (reported, all ranks fall back together)
        h, err = None, f"gs_exchange_handle: {e}"
    parts = [None] * world
    dist.all_gather_object(parts, h, group=group)
    if not err and any(p is None for p in parts):
        err = "another rank could not export its buffer"
    if not err:
        try:
            ctx.exchange_open(parts, rank)
            ctx.synchronize()
        except Exception as e:  # noqa: BLE001
            err = f"gs_exchange_open: {e}"
    ok = torch.tensor([0 if err else 1], dtype=torch.int64)
    dist.all_reduce(ok, group=group)
    if int(ok.item()) != world:
        if not err:
            err = "another rank could not open the exchange"
            ctx.exchange_close()
        return err
    return ""


class ShardedSampler:
    """A Context holding this rank's shard, joined to the other ranks over RCCL."""

    def __init__(self, codes: np.ndarray, offsets: np.ndarray, alphabet: bytes, rank: int,
                 world: int, device: int, group=None, bounds=None, exchange: bool = False):
        from ._native import Context
        lengths = np.diff(np.asarray(offsets, np.int64))
        self.bounds = bounds or shard_bounds(lengths, world)
        lo, hi = self.bounds[rank]
        self.lo, self.hi, self.rank, self.world = lo, hi, rank, world
        o = np.asarray(offsets, np.int64)
        self.ctx = Context(device)
        self.ctx.set_sequences(np.asarray(codes, np.uint8)[o[lo]:o[hi]], o[lo:hi + 1] - o[lo],
                               alphabet, n_global=len(lengths), global_offset=lo)
        if world > 1:
            self.ctx.comm_init(exchange_unique_id(rank, group), world, rank)
        self.exchange_error = open_exchange(self.ctx, rank, world, group) if exchange else None

    def set_positions(self, W: int, pos_global: np.ndarray) -> None:
        self.ctx.set_positions(W, np.asarray(pos_global, np.int32)[self.lo:self.hi])

    def run_sweeps(self, pc: float, cutoff: float, n: int, seed: int, first: int = 0) -> None:
        self.ctx.run_sweeps(pc, cutoff, n, seed, first)

    def gather_state(self, group=None):
        """All ranks' (positions, PWMS) in global order, on every rank."""
        import torch.distributed as dist
        pos, pw = self.ctx.get_state()
        if self.world == 1:
            return pos, pw
        parts = [None] * self.world
        dist.all_gather_object(parts, (pos, pw), group=group)
        return (np.concatenate([p for p, _ in parts]), np.concatenate([w for _, w in parts]))
