"""Multi-GPU sharding of independent QP instances (one process per GPU).

QP instances share nothing, so the hot path shards with no collective at all: rank r solves
the contiguous slice [r*B/G, (r+1)*B/G).  When one rank owns the
whole input batch (a simulator on rank 0), ``scatter_batch`` / ``gather_solutions`` move the
input stacks out and the primal solutions back with one collective each -- torch.distributed
over RCCL ("nccl" backend on ROCm, xGMI) for device tensors, gloo for host tensors in tests.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

FIELDS = ("Ad", "Bd", "gd", "x0", "xref", "contact")


def shard_bounds(B: int, rank: int, world: int):
    """Contiguous, balanced slice [lo, hi) of B instances for `rank` of `world`."""
    base, rem = divmod(B, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def shard_batch(batch: dict, rank: int, world: int) -> dict:
    B = batch["Ad"].shape[0]
    lo, hi = shard_bounds(B, rank, world)
    return {k: batch[k][lo:hi] for k in FIELDS}


def _pad_chunks(t: torch.Tensor, world: int):
    B = t.shape[0]
    per = (B + world - 1) // world
    chunks = []
    for r in range(world):
        lo, hi = shard_bounds(B, r, world)
        c = t[lo:hi]
        if c.shape[0] < per:
            c = torch.cat([c, c.new_zeros((per - c.shape[0],) + tuple(t.shape[1:]))], 0)
        chunks.append(c.contiguous())
    return chunks, per


def scatter_batch(batch: dict | None, B: int, N: int, device, group=None) -> dict:
    """Rank 0 holds `batch` (tensors on `device`); every rank receives its shard.  All ranks
    pass the global B and horizon N."""
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    lo, hi = shard_bounds(B, rank, world)
    per = (B + world - 1) // world
    shapes = {"Ad": (12, 12), "Bd": (N, 12, 12), "gd": (12,), "x0": (12,), "xref": (N, 12),
              "contact": (4, N)}
    out = {}
    for k in FIELDS:
        dt = torch.uint8 if k == "contact" else torch.float32
        recv = torch.empty((per,) + shapes[k], dtype=dt, device=device)
        if rank == 0:
            chunks, _ = _pad_chunks(batch[k], world)
            dist.scatter(recv, chunks, src=0, group=group)
        else:
            dist.scatter(recv, None, src=0, group=group)
        out[k] = recv[: hi - lo]
    return out


def gather_solutions(w_local: torch.Tensor, B: int, group=None):
    """Gather each rank's (B_r, 24N) primal block to rank 0 -> (B, 24N) on rank 0, None
    elsewhere."""
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    per = (B + world - 1) // world
    pad = w_local
    if w_local.shape[0] < per:
        pad = torch.cat([w_local, w_local.new_zeros((per - w_local.shape[0],) + tuple(w_local.shape[1:]))], 0)
    pad = pad.contiguous()
    if rank == 0:
        bufs = [torch.empty_like(pad) for _ in range(world)]
        dist.gather(pad, bufs, dst=0, group=group)
        parts = []
        for r in range(world):
            lo, hi = shard_bounds(B, r, world)
            parts.append(bufs[r][: hi - lo])
        return torch.cat(parts, 0)
    dist.gather(pad, None, dst=0, group=group)
    return None
