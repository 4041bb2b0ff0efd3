"""GPU diagnostic: per-tensor errors of the Atari and MLP paths vs the oracle (no asserts)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as orc  # noqa: E402
from freeimpala_amd.learner import DeviceLearner  # noqa: E402


def bf(u):
    return (np.asarray(u, np.uint16).astype(np.uint32) << 16).view(np.float32)


def err(a, b):
    a = np.asarray(a, np.float64).ravel()
    b = np.asarray(b, np.float64).ravel()
    d = np.abs(a - b)
    i = int(d.argmax())
    return (f"relL2 {np.linalg.norm(a - b) / max(1e-30, np.linalg.norm(b)):.2e} scmax {d.max() / max(1e-30, np.abs(b).max()):.2e}"
            f" at {i} gpu {a[i]:.6g} ref {b[i]:.6g} |ref|max {np.abs(b).max():.4g} ratio(sum) {a.sum() / (b.sum() + 1e-30):.6f}")


def atari(T, B):
    A = 18
    L = DeviceLearner("atari", seq_len=T, batch=B, num_actions=A, optimizer="sgd", lr=1e-3, max_grad_norm=0.0)
    L.synth(seed=T * 100 + B)
    N = (T + 1) * B
    fr = L.tensor("frames", np.uint8, (N, 84, 84, 4))
    p0 = L.get_params()
    L.step_resident()
    acts = orc.atari_forward(fr, p0, A=A, bf16_emul=True)
    print(f"== atari T={T} B={B} N={N}")
    for nm, sh in [("a1", (N, 20, 20, 32)), ("a2", (N, 9, 9, 64)), ("a3", (N, 7, 7, 64)), ("h", (N, 512))]:
        print(nm, err(bf(L.tensor(nm, np.uint16, sh)), orc.bf16_round(acts[nm])))
    dl = L.tensor("dlogits", shape=(T, B, A))
    dv = L.tensor("dvalue", shape=(T + 1, B))
    dout = np.zeros((N, A + 1), np.float32)
    dout[:T * B, :A] = dl.reshape(T * B, A)
    dout[:, A] = dv.reshape(N)
    g_ref, mids = orc.atari_backward_ex(fr, p0, acts, dout, A=A, bf16_emul=True)
    for nm, key, sh in [("dh", "dh", (N, 512)), ("da3", "d3", (N, 7, 7, 64)), ("da2", "d2", (N, 9, 9, 64)),
                        ("da1", "d1", (N, 20, 20, 32))]:
        print(nm, err(bf(L.tensor(nm, np.uint16, sh)), orc.bf16_round(mids[key])))
    g = L.tensor("grads")
    sizes = [8192, 32, 32768, 64, 36864, 64, 3136 * 512, 512, 512 * (A + 1), A + 1]
    off = np.cumsum([0] + sizes)
    for i, nm in enumerate(["c1W", "c1b", "c2W", "c2b", "c3W", "c3b", "fcW", "fcb", "hW", "hb"]):
        print(nm, err(g[off[i]:off[i + 1]], g_ref[off[i]:off[i + 1]]))


def mlp(T, B):
    A, D, H = 18, 128, 256
    L = DeviceLearner("mlp", seq_len=T, batch=B, num_actions=A, optimizer="sgd", lr=1e-3, max_grad_norm=0.0)
    L.synth(seed=42)
    batch = orc.synth_batch(42, T=T, B=B, A=A, D=D)
    p0 = L.get_params()
    L.step_resident()
    obs = batch["obs"].reshape(-1, D)
    h1, h2, out = orc.mlp_forward(obs, p0, H=H, A=A)
    print(f"== mlp T={T} B={B}")
    print("h1", err(L.tensor("h1"), h1))
    print("h2", err(L.tensor("h2"), h2))
    dl = L.tensor("dlogits", shape=(T, B, A))
    dv = L.tensor("dvalue", shape=(T + 1, B))
    dout = np.zeros(((T + 1) * B, A + 1), np.float32)
    dout[:T * B, :A] = dl.reshape(T * B, A)
    dout[:, A] = dv.reshape(-1)
    g_ref = orc.mlp_backward(obs, p0, h1, h2, dout, H=H, A=A)
    g = L.tensor("grads")
    off = np.cumsum([0, D * H, H, H * H, H, H * (A + 1), A + 1])
    for i, nm in enumerate(["W1", "b1", "W2", "b2", "Wh", "bh"]):
        print(nm, err(g[off[i]:off[i + 1]], g_ref[off[i]:off[i + 1]]))


if __name__ == "__main__":
    atari(2, 16)
    atari(3, 32)
    mlp(100, 512)
    mlp(20, 48)
