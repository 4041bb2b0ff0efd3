"""Generate tests/golden/farmer_*.npz from the REFERENCE's own FarmerLstmModel.

Run in the build container only (it imports /root/reference/scripts/gpu_benchmark.py, which
does not exist on the GPU box):  python tests/golden/make_farmer_golden.py

For each case the reference model (gpu_benchmark.FarmerLstmModel, :11-44) is built, its
parameters are overwritten with oracle/farmer_oracle.gen_params(seed) (so the fixture needs no
parameter dump), and the reference train step (gpu_benchmark.run_single_training_iteration,
:99-125, with get_loss_function / get_optimizer, :46-66) runs STEPS times on fixed inputs.
Stored per step: the forward value, the loss, every gradient (full for tensors of <= 4096
elements; for larger ones the sum, the sum of squares and NSAMP elements at fixed indices) and
the parameters after the optimizer step (same reduction).
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, "/root/reference/scripts")
import gpu_benchmark as ref  # noqa: E402  (the reference)

from oracle import farmer_oracle as fo  # noqa: E402

NSAMP = 1024
STEPS = 2
CASES = [  # name, B, T, loss, optimizer, lr, param seed, input seed
    ("farmer_b4_t5_mse_adam", 4, 5, "mse", "adam", 1e-3, 1, 11),
    ("farmer_b32_t10_mse_adam", 32, 10, "mse", "adam", 1e-3, 2, 12),  # gpu_benchmark defaults
    ("farmer_b8_t7_huber_adamw", 8, 7, "huber", "adamw", 1e-3, 3, 13),
    ("farmer_b6_t3_mae_sgd", 6, 3, "mae", "sgd", 1e-2, 4, 14),
]


def sample_idx(n, seed=123):
    return np.sort(np.random.RandomState(seed + n).choice(n, NSAMP, replace=False)) if n > 4096 else None


def reduce(name, a, out, prefix):
    a = np.array(a, np.float32, copy=True).reshape(-1)  # never a view of a live torch tensor
    idx = sample_idx(a.size)
    if idx is None:
        out[f"{prefix}/{name}"] = a
    else:
        out[f"{prefix}/{name}:idx"] = idx
        out[f"{prefix}/{name}:val"] = a[idx]
        out[f"{prefix}/{name}:sum"] = np.float64(a.astype(np.float64).sum())
        out[f"{prefix}/{name}:sumsq"] = np.float64((a.astype(np.float64) ** 2).sum())


def main():
    torch.set_num_threads(4)
    torch.manual_seed(0)
    gdir = os.path.dirname(os.path.abspath(__file__))
    for name, B, T, loss, opt, lr, ps, xs in CASES:
        model = ref.FarmerLstmModel()
        names = [n for n, _ in model.named_parameters()]
        assert names == [n for n, _ in fo.SHAPES], names
        p0 = fo.gen_params(ps)
        with torch.no_grad():
            for n, (a, b, s) in fo.offsets().items():
                dict(model.named_parameters())[n].copy_(torch.from_numpy(p0[a:b].reshape(s)))
        z, x, y = fo.gen_inputs(xs, B, T)
        zt, xt, yt = (torch.from_numpy(v) for v in (z, x, y))
        crit = ref.get_loss_function(loss)
        optim = ref.get_optimizer(opt, model.parameters(), lr)
        out = {"B": B, "T": T, "loss_kind": loss, "optimizer": opt, "lr": lr, "param_seed": ps,
               "input_seed": xs, "z": z, "x": x, "y": y, "steps": STEPS}
        for s in range(STEPS):
            with torch.no_grad():
                val = model(zt, xt, return_value=True)["values"].numpy().copy()
            _, lv = ref.run_single_training_iteration(model, zt, xt, yt, crit, optim, torch.device("cpu"))
            out[f"step{s}/value"] = val
            out[f"step{s}/loss"] = np.float64(lv)
            for n, prm in model.named_parameters():
                reduce(n, prm.grad.numpy(), out, f"step{s}/grad")
                reduce(n, prm.detach().numpy(), out, f"step{s}/param")
        np.savez_compressed(os.path.join(gdir, name + ".npz"), **out)
        print(name, "loss", [float(out[f"step{s}/loss"]) for s in range(STEPS)])


if __name__ == "__main__":
    main()
