"""One rank of the two-process data-parallel check (tests/test_gpu_learner.py::
test_two_process_attach_comm_matches_single_device): bench.py's N > 1 path without the timing.

Launched as `python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 ...
tests/dist_attach_worker.py --arch {mlp,atari} --out DIR`, one rank per device (LOCAL_RANK).
Each rank owns columns [rank*B/N, (rank+1)*B/N) of the global synthetic batch,
gets the RCCL unique id from rank 0 over gloo (freeimpala_amd.launch.broadcast_bytes), attaches
its handle (fi_learner_attach_comm) and runs SGD steps with the in-step bucketed all-reduce.
The ranks' parameters are gathered over gloo; rank 0 also steps the WHOLE batch on one device
and writes result.json: replicas bit-identical, and their distance to the one-device run.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="mlp")
    ap.add_argument("--out", required=True)
    ap.add_argument("--steps", type=int, default=2)
    args = ap.parse_args()
    rank, ws, local = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"]), int(os.environ["LOCAL_RANK"])
    from freeimpala_amd import _abi
    _abi.lib()  # the learner library before torch (bench.py's order)
    import torch
    import torch.distributed as dist
    from freeimpala_amd.launch import broadcast_bytes, shard_columns
    from freeimpala_amd.learner import DeviceLearner
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    T, B = (4, 64) if args.arch == "mlp" else (2, 32)
    bl = B // ws
    kw = dict(seq_len=T, num_actions=18, optimizer="sgd", lr=1e-3, max_grad_norm=0.0, seed=6)
    L = DeviceLearner(args.arch, batch=bl, device=local, **kw)
    off, _ = shard_columns(rank, ws, bl)
    L.synth(seed=12, b_global=B, b_offset=off)
    uid = broadcast_bytes(DeviceLearner.comm_unique_id() if rank == 0 else b"", 0)
    L.attach_comm(uid, rank, ws)
    info = L.comm_info()
    losses = [L.step_resident()["total_loss"] for _ in range(args.steps)]
    p = torch.from_numpy(L.get_params().copy())
    gathered = [torch.zeros_like(p) for _ in range(ws)]
    dist.all_gather(gathered, p)
    lt = torch.tensor(losses, dtype=torch.float64)
    dist.all_reduce(lt)  # sum of the shards' losses = the full batch's (losses are sums)
    if rank == 0:
        full = DeviceLearner(args.arch, batch=B, device=local, **kw)
        full.synth(seed=12, b_global=B, b_offset=0)
        full_losses = [full.step_resident()["total_loss"] for _ in range(args.steps)]
        pf = full.get_params().astype(np.float64)
        reps = [g.numpy() for g in gathered]
        scale = max(1.0, float(np.abs(pf).max()))
        res = {
            "world": ws,
            "comm": info,
            "buckets_last_step": L.comm_info()["buckets_last_step"],
            "replicas_identical": all(np.array_equal(reps[0], r) for r in reps[1:]),
            "max_scaled_diff_vs_one_device": float(np.abs(reps[0] - pf).max()) / scale,
            "loss_sum": lt.tolist(),
            "one_device_loss": full_losses,
        }
        with open(os.path.join(args.out, "result.json"), "w") as f:
            json.dump(res, f)
        full.close()
    L.close()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
