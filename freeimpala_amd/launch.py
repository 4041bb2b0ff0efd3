"""Launcher-side plumbing of the data-parallel learner (one process per GPU).

SURVEY.md 8(e): rank g of N owns batch columns [g*B, (g+1)*B) of the global batch (weak
scaling, B per GPU); the only exchange inside the step is the RCCL all-reduce of the flat
gradient, done by the C ABI on the learner stream. What the launcher does around it lives
here so that it can be exercised on CPU with the gloo backend (tests/test_dist_gloo.py):
  * shard_columns       -- the column range of a rank;
  * broadcast_bytes     -- the RCCL unique id from rank 0 to every rank (gloo tensors);
  * max_over_ranks      -- the bench's max-over-ranks wall time;
  * split_entries       -- a SharedBuffer::readBatch result (M host entries) split into the
                           N contiguous per-GPU shards (reference data_structures.h:267-300).
torch.distributed is plumbing only; the product math never goes through it.
"""
from __future__ import annotations

from typing import Sequence


def shard_columns(rank: int, world: int, b_per_rank: int) -> tuple[int, int]:
    """(first global column, count) of `rank` under weak scaling."""
    if not (0 <= rank < world) or b_per_rank <= 0:
        raise ValueError(f"bad shard rank={rank} world={world} B={b_per_rank}")
    return rank * b_per_rank, b_per_rank


def split_entries(entries: Sequence, world: int) -> list:
    """M entries -> world contiguous shards of M/world entries each (M % world == 0)."""
    m = len(entries)
    if world <= 0 or m % world:
        raise ValueError(f"{m} entries do not split evenly over {world} ranks")
    k = m // world
    return [list(entries[r * k:(r + 1) * k]) for r in range(world)]


def broadcast_bytes(blob: bytes, src: int = 0) -> bytes:
    """Broadcast a byte string from `src` over the default process group (gloo)."""
    import torch
    import torch.distributed as dist
    rank = dist.get_rank()
    size = torch.tensor([len(blob) if rank == src else 0], dtype=torch.int64)
    dist.broadcast(size, src)
    buf = torch.zeros(int(size.item()), dtype=torch.uint8)
    if rank == src and len(blob):
        buf[:] = torch.frombuffer(bytearray(blob), dtype=torch.uint8)
    dist.broadcast(buf, src)
    return buf.numpy().tobytes()


def max_over_ranks(x: float) -> float:
    import torch
    import torch.distributed as dist
    t = torch.tensor([float(x)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
