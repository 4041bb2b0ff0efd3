"""Launcher-side plumbing of the data-parallel learner (one process per GPU).

SURVEY.md 8(e): rank g of N owns batch columns [g*B, (g+1)*B) of the global batch (weak
scaling, B per GPU); the only exchange inside the step is the RCCL all-reduce of the flat
gradient, done by the C ABI on the learner stream. What the launcher does around it lives
here so that it can be exercised on CPU with the gloo backend (tests/test_dist_gloo.py):
  * shard_columns       -- the column range of a rank;
  * broadcast_bytes     -- the RCCL unique id from rank 0 to every rank (gloo tensors);
  * max_over_ranks      -- the bench's max-over-ranks wall time;
  * split_entries       -- a SharedBuffer::readBatch result (M host entries) split into the
                           N contiguous per-GPU shards (reference data_structures.h:267-300);
  * gather_objects / data_parallel_fields -- bench.py's N > 1 line: every rank's own ms/step,
                           its exposed all-reduce wait and the bytes all-reduced per step, so a
                           scaling run explains itself (weak-scaling loss vs exposed exchange);
  * bench_launch_plan   -- `python bench.py --gpus N` without a launcher: the torch.distributed.run
                           command that starts the N ranks (decided before anything touches the GPU);
  * timed_steps         -- the timed loop: a rank's own time and the barrier-bracketed time.
torch.distributed is plumbing only; the product math never goes through it.
"""
from __future__ import annotations

import time
from typing import Callable, Mapping, Sequence

# environment a torch.distributed launcher sets in every rank it starts
LAUNCHER_ENV = ("WORLD_SIZE", "LOCAL_RANK", "TORCHELASTIC_RUN_ID")


class LaunchError(RuntimeError):
    """bench.py was asked for a GPU count it cannot honour."""


def bench_launch_plan(gpus: int, env: Mapping[str, str], argv: Sequence[str], script: str,
                      python: str, visible_devices: Callable[[], int], port: int) -> list | None:
    """How bench.py runs for `--gpus N` (BASELINE metric: 1/2/4/8 MI355X, one process per GPU).

    Returns None when this process is one of the ranks already (N == 1, or started by a
    launcher whose WORLD_SIZE equals N), else the command of the child launcher that starts N
    ranks of the same script with the same arguments; the caller runs it as a child process and
    exits with its code (never an exec: the parent has not touched the GPU, and must not).
    Raises LaunchError when --gpus disagrees with the launcher's WORLD_SIZE, or when fewer than N
    devices are visible (FI_BENCH_DEVICE, the one-device rehearsal that pins every rank to one
    device, needs one). `visible_devices` is only called when ranks must be started."""
    if gpus < 1:
        raise LaunchError(f"--gpus must be >= 1 (got {gpus})")
    if any(k in env for k in LAUNCHER_ENV):
        ws = int(env.get("WORLD_SIZE", "1"))
        if ws != gpus:
            raise LaunchError(f"--gpus {gpus} disagrees with the launcher's WORLD_SIZE={ws}")
        return None
    if gpus == 1:
        return None
    need = 1 if env.get("FI_BENCH_DEVICE") not in (None, "") else gpus
    have = int(visible_devices())
    if have < need:
        raise LaunchError(f"--gpus {gpus} needs {need} visible GPU(s), {have} visible")
    return [python, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", script, *argv]


def timed_steps(step: Callable[[], object], sync: Callable[[], object], barrier: Callable[[], object],
                steps: int) -> tuple[float, float]:
    """(own, bracketed) seconds for `steps` steps. Both start after a barrier; `own` stops when
    this rank's device work has drained (before the closing barrier, so it is this rank's time
    alone); `bracketed` stops after the closing barrier (what the max over ranks is taken of)."""
    barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    own = time.perf_counter() - t0
    barrier()
    return own, time.perf_counter() - t0


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


def gather_objects(obj) -> list:
    """Every rank's `obj` (a small picklable dict), in rank order, on every rank (gloo)."""
    import torch.distributed as dist
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj)
    return out


def data_parallel_fields(per_rank: Sequence[dict], grad_bytes: int, buckets: int | None) -> dict:
    """The N > 1 fields of bench.py's line from every rank's own measurements.

    per_rank[r] = {"ms_per_step": the rank's own timed-loop ms/step (its device work drained,
                                  before the closing barrier and the max over ranks),
                   "allreduce_ms": the rank's exposed all-reduce wait per step (the learner's
                   "allreduce" phase: the compute stream waiting for buckets still in flight
                   after the backward, HIP events over the profiled steps)}.
    grad_bytes: the flat fp32 gradient all-reduced once per step (+ the 4-byte reject flag).
    A ring all-reduce moves 2 (N - 1) / N of the buffer over each rank's links."""
    n = len(per_rank)
    ms = [float(d["ms_per_step"]) for d in per_rank]
    ar = [float(d["allreduce_ms"]) for d in per_rank]
    payload = int(grad_bytes) + 4
    return {
        "ranks": n,
        "allreduce_bytes_per_step": payload,
        "allreduce_ring_bytes_per_rank_per_step": int(round(2 * (n - 1) / n * payload)) if n else 0,
        "allreduce_buckets_per_step": buckets,
        "exposed_allreduce_ms": {"max": round(max(ar), 5), "mean": round(sum(ar) / n, 5),
                                 "per_rank": [round(x, 5) for x in ar]},
        "rank_ms_per_step": {"max": round(max(ms), 4), "mean": round(sum(ms) / n, 4),
                             "min": round(min(ms), 4), "per_rank": [round(x, 4) for x in ms]},
    }
