"""The torch-CPU learner that bench.py times as `cpu_baseline` computes the oracle's step:
same parameter layout, same V-trace / loss, same gradients (fp32 oneDNN vs the oracle's fp64
accumulation, so compared by relative L2). CPU only."""
import numpy as np
import pytest


def _ref_grads(orc, arch, batch, p, A, D=16, H=32):
    T, B = batch["actions"].shape
    if arch == "mlp":
        obs = batch["obs"].reshape(-1, D)
        h1, h2, out = orc.mlp_forward(obs, p, H=H, A=A)
    else:
        fr = batch["frames"].reshape(-1, 84, 84, 4)
        acts = orc.atari_forward(fr, p, A=A, bf16_emul=False)
        out = acts["out"]
    vt = orc.vtrace_loss(out[:, :A].reshape(T + 1, B, A)[:T], batch["mu"], batch["actions"],
                         batch["rewards"], batch["discounts"], out[:, A].reshape(T + 1, B))
    dout = np.zeros(((T + 1) * B, A + 1), np.float32)
    dout[:T * B, :A] = vt["dlogits"].reshape(T * B, A)
    dout[:, A] = vt["dvalue"].reshape(-1)
    if arch == "mlp":
        g = orc.mlp_backward(obs, p, h1, h2, dout, H=H, A=A)
    else:
        g = orc.atari_backward(fr, p, acts, dout, A=A, bf16_emul=False)
    return g, vt["losses"]


@pytest.mark.parametrize("arch", ["mlp", "atari"])
def test_torch_cpu_learner_matches_oracle(orc, arch):
    torch = pytest.importorskip("torch")
    from oracle.torch_learner import TorchLearner
    A, D, H = 6, 16, 32
    T, B = (5, 8) if arch == "mlp" else (2, 3)
    batch = orc.synth_batch(9, T=T, B=B, A=A, D=D, obs=arch == "mlp", frames=arch == "atari")
    n = orc.mlp_param_count(D, H, A) if arch == "mlp" else orc.atari_param_count(A)
    p = np.random.RandomState(3).uniform(-0.1, 0.1, n).astype(np.float32)
    g_ref, l_ref = _ref_grads(orc, arch, batch, p, A, D, H)
    tl = TorchLearner(arch, p, A=A, D=D, H=H)
    g, losses = tl.grads(batch)
    g = g.numpy().astype(np.float64)
    rel = np.linalg.norm(g - g_ref) / np.linalg.norm(g_ref)
    assert rel < 1e-4, rel
    np.testing.assert_allclose(losses, l_ref, rtol=1e-4, atol=1e-4)
    # one Adam step with the clip equals the oracle's clip + adam on the same gradient
    g32 = g_ref.astype(np.float32).copy()
    orc.clip_grad_norm(g32, 40.0)
    pr, m, v = p.copy(), np.zeros_like(p), np.zeros_like(p)
    orc.adam(pr, g32, m, v, 5e-4, 0.9, 0.999, 1e-8, 1)
    tl.step(batch)
    assert np.abs(tl.p.numpy() - pr).max() <= 1e-5 + 1e-3 * np.abs(pr - p).max()
    del torch
