"""Data-parallel path on CPU: world_size 2 with the gloo backend.

Each rank owns batch columns [r*B, (r+1)*B) of the global synthetic batch; losses are sums,
so the sum-all-reduce of the per-shard gradients must equal the gradient of the
concatenated batch (rel 1e-5, the multi-GPU parity bar of SURVEY.md 8(c)). The gradients
here come from the CPU oracle (the HIP path does the same all-reduce with RCCL inside
fi_learner_step; its GPU test is test_gpu_learner.py); this covers the launcher logic
(freeimpala_amd/launch.py) the bench uses at N > 1: shard ranges, unique-id broadcast,
max-over-ranks timing, the entry split of a readBatch result.
"""
import os
import socket

import numpy as np
import pytest


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, T, B, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    from freeimpala_amd import launch
    from oracle import oracle as orc
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        D, H, A = 32, 64, 6
        b0, nb = launch.shard_columns(rank, world, B)
        batch = orc.synth_batch(42, T=T, B=nb, A=A, D=D, B_glob=world * B, b_off=b0)
        p = np.random.RandomState(0).uniform(-0.1, 0.1, orc.mlp_param_count(D, H, A)).astype(np.float32)
        obs = batch["obs"].reshape((T + 1) * nb, D)
        h1, h2, out = orc.mlp_forward(obs, p, H=H, A=A)
        logits = out[:, :A].reshape(T + 1, nb, A)
        values = out[:, A].reshape(T + 1, nb)
        vt = orc.vtrace_loss(logits[:T], batch["mu"], batch["actions"], batch["rewards"],
                             batch["discounts"], values)
        dout = np.zeros(((T + 1) * nb, A + 1), np.float32)
        dout[:T * nb, :A] = vt["dlogits"].reshape(T * nb, A)
        dout[:, A] = vt["dvalue"].reshape(-1)
        g = torch.from_numpy(orc.mlp_backward(obs, p, h1, h2, dout, H=H, A=A))
        dist.all_reduce(g)  # the exchange step (RCCL ncclAllReduce(sum) on the GPUs)
        loss = torch.tensor(vt["losses"], dtype=torch.float64)
        dist.all_reduce(loss)
        uid = launch.broadcast_bytes(bytes(range(7, 7 + 128)) if rank == 0 else b"", 0)
        tmax = launch.max_over_ranks(1.5 + rank)
        if rank == 0:
            np.save(os.path.join(out_dir, "g.npy"), g.numpy())
            np.save(os.path.join(out_dir, "loss.npy"), loss.numpy())
        np.save(os.path.join(out_dir, f"meta{rank}.npy"),
                np.array([b0, nb, tmax, len(uid), uid == bytes(range(7, 7 + 128))], np.float64))
    finally:
        dist.destroy_process_group()


def test_dp_allreduce_equals_concatenated_batch(tmp_path, orc):
    import torch.multiprocessing as mp
    T, B, world = 6, 8, 2
    mp.start_processes(_worker, args=(world, _free_port(), T, B, str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    # single "device" on the concatenated batch
    D, H, A = 32, 64, 6
    full = orc.synth_batch(42, T=T, B=world * B, A=A, D=D)
    p = np.random.RandomState(0).uniform(-0.1, 0.1, orc.mlp_param_count(D, H, A)).astype(np.float32)
    obs = full["obs"].reshape((T + 1) * world * B, D)
    h1, h2, out = orc.mlp_forward(obs, p, H=H, A=A)
    logits = out[:, :A].reshape(T + 1, world * B, A)
    values = out[:, A].reshape(T + 1, world * B)
    vt = orc.vtrace_loss(logits[:T], full["mu"], full["actions"], full["rewards"], full["discounts"], values)
    dout = np.zeros(((T + 1) * world * B, A + 1), np.float32)
    dout[:T * world * B, :A] = vt["dlogits"].reshape(-1, A)
    dout[:, A] = vt["dvalue"].reshape(-1)
    g_full = orc.mlp_backward(obs, p, h1, h2, dout, H=H, A=A).astype(np.float64)
    g_dp = np.load(tmp_path / "g.npy").astype(np.float64)
    assert np.linalg.norm(g_dp - g_full) <= 1e-5 * np.linalg.norm(g_full)
    np.testing.assert_allclose(np.load(tmp_path / "loss.npy"), vt["losses"], rtol=1e-9, atol=1e-9)
    for r in range(world):
        b0, nb, tmax, nuid, same = np.load(tmp_path / f"meta{r}.npy")
        assert (b0, nb) == (r * B, B)
        assert tmax == 1.5 + world - 1 and nuid == 128 and same == 1


def test_split_entries_and_shards():
    from freeimpala_amd import launch
    entries = [bytes([i]) * 4 for i in range(8)]
    sh = launch.split_entries(entries, 4)
    assert [len(s) for s in sh] == [2] * 4 and sh[3][1] == entries[7]
    with pytest.raises(ValueError):
        launch.split_entries(entries, 3)
    assert launch.shard_columns(3, 8, 4096) == (3 * 4096, 4096)
    with pytest.raises(ValueError):
        launch.shard_columns(8, 8, 4096)


def _dp_fields_worker(rank, world, port, out_dir):
    """bench.py's N > 1 reporting as it runs under torch.distributed.run (FI_BENCH_NO_COMM
    rehearsal on CPU): each rank contributes its own ms/step and exposed all-reduce wait, every
    rank gathers all of them and builds the line's data_parallel object."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import json
    import torch.distributed as dist
    from freeimpala_amd import launch
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        own = {"ms_per_step": 24.0 + rank, "allreduce_ms": 0.1 * (rank + 1)}
        per = launch.gather_objects(own)
        dp = launch.data_parallel_fields(per, grad_bytes=4 * 1693875, buckets=3)
        with open(os.path.join(out_dir, f"dp{rank}.json"), "w") as fh:
            json.dump(dp, fh)
    finally:
        dist.destroy_process_group()


def test_bench_data_parallel_fields_world2(tmp_path):
    """bench.py's N > 1 line carries the bytes all-reduced per step, the exposed
    all-reduce wait per rank (max / mean) and every rank's own ms/step, gathered over gloo."""
    import json
    import torch.multiprocessing as mp
    world = 2
    mp.start_processes(_dp_fields_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    dps = [json.load(open(tmp_path / f"dp{r}.json")) for r in range(world)]
    assert dps[0] == dps[1]  # every rank holds the same gathered view
    dp = dps[0]
    assert dp["ranks"] == 2
    assert dp["allreduce_bytes_per_step"] == 4 * 1693875 + 4
    assert dp["allreduce_ring_bytes_per_rank_per_step"] == 4 * 1693875 + 4  # 2 (N-1)/N = 1 at N = 2
    assert dp["allreduce_buckets_per_step"] == 3
    assert dp["rank_ms_per_step"]["per_rank"] == [24.0, 25.0] and dp["rank_ms_per_step"]["max"] == 25.0
    assert dp["exposed_allreduce_ms"] == {"max": 0.2, "mean": 0.15, "per_rank": [0.1, 0.2]}
