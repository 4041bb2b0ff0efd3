"""The torch-CPU FarmerLstm port timed as scripts/farmer_bench.py's CPU baseline computes the
same gradients as the fp64 oracle (itself pinned to the reference's golden vectors)."""
import numpy as np


def test_torch_port_gradients_match_oracle():
    import torch
    from oracle import farmer_oracle as fo
    from oracle.farmer_torch import TorchFarmer
    p0 = fo.gen_params(7)
    z, x, y = fo.gen_inputs(8, 6, 9)
    tf = TorchFarmer(p0, "huber", "sgd", 1e-2)
    tf.step(*(torch.from_numpy(a) for a in (z, x, y)))
    v, saved = fo.forward(p0, z, x)
    _, dv = fo.loss_and_grad(v, y, "huber")
    g = fo.backward(p0, saved, dv)
    gt = tf.grads()
    for n, (a, b, s) in fo.offsets().items():
        d = np.linalg.norm(gt[a:b] - g[a:b])
        assert d <= 1e-5 * np.linalg.norm(g[a:b]) + 1e-7 * np.sqrt(b - a), n
