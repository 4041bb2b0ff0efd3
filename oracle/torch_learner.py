"""TEST INFRASTRUCTURE / CPU BASELINE ONLY -- never imported by the product path.

The same IMPALA learner step as oracle/impala_oracle.c (policy forward -> V-trace + loss ->
backward -> global-norm clip -> Adam), written on PyTorch's CPU kernels (oneDNN / MKL
convolutions and GEMMs, fp32, multithreaded), so bench.py's `cpu_baseline` is timed on an
optimised CPU learner rather than on the oracle's scalar fp64 loops. The reference's own
learner-side numerics live on the same stack (libtorch / PyTorch:
/root/reference/cmd/libtorch_bench/main.cpp:14-42, scripts/gpu_benchmark.py:11-60).

Parameter blob layout = the oracle's / the product's:
  MLP    W1[D][H] b1 W2[H][H] b2 Wh[H][A+1] bh
  Atari  c1W[8][8][4][32] c1b c2W[4][4][32][64] c2b c3W[3][3][64][64] c3b fcW[3136][512] fcb
         hW[512][A+1] hb            (NHWC activations, frames u8 scaled by 1/255)
The gradients equal the oracle's (tests/test_torch_baseline.py, fp32 vs fp64 tolerance).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

HP = dict(rho_bar=1.0, c_bar=1.0, pg_rho_bar=1.0, lambda_=1.0, baseline_cost=0.5,
          entropy_cost=0.01)


def _views(p: torch.Tensor, shapes):
    out, o = [], 0
    for s in shapes:
        n = int(np.prod(s))
        out.append(p[o:o + n].view(*s))
        o += n
    assert o == p.numel(), (o, p.numel())
    return out


def mlp_shapes(D, H, A):
    return [(D, H), (H,), (H, H), (H,), (H, A + 1), (A + 1,)]


def atari_shapes(A):
    return [(8, 8, 4, 32), (32,), (4, 4, 32, 64), (64,), (3, 3, 64, 64), (64,), (3136, 512),
            (512,), (512, A + 1), (A + 1,)]


def mlp_forward(p, obs, D, H, A):
    W1, b1, W2, b2, Wh, bh = _views(p, mlp_shapes(D, H, A))
    h1 = torch.relu(obs @ W1 + b1)
    h2 = torch.relu(h1 @ W2 + b2)
    return h2 @ Wh + bh


def atari_forward(p, frames_u8, A):
    """frames (N,84,84,4) uint8 NHWC -> (N, A+1)."""
    c1W, c1b, c2W, c2b, c3W, c3b, fcW, fcb, hW, hb = _views(p, atari_shapes(A))
    x = frames_u8.permute(0, 3, 1, 2).float()  # NCHW, integers
    conv = lambda x, W, b, s: F.conv2d(x, W.permute(3, 2, 0, 1), b, stride=s)
    a1 = torch.relu(conv(x, c1W, None, 4) * (1.0 / 255.0) + c1b.view(1, -1, 1, 1))
    a2 = torch.relu(conv(a1, c2W, c2b, 2))
    a3 = torch.relu(conv(a2, c3W, c3b, 1))
    flat = a3.permute(0, 2, 3, 1).reshape(a3.shape[0], 3136)  # NHWC flatten order
    h = torch.relu(flat @ fcW + fcb)
    return h @ hW + hb


def vtrace_loss(logits, mu, actions, rewards, discounts, values, hp=HP):
    """IMPALA eq. 1 / section 4.2 as in oracle/impala_oracle.c (sums over T*B).
    logits (T,B,A) with grad, values (T+1,B) with grad; returns (total, (pg, base, ent))."""
    T = logits.shape[0]
    logp = torch.log_softmax(logits, -1)
    with torch.no_grad():
        lmu = torch.log_softmax(mu, -1)
        a = actions.long().unsqueeze(-1)
        log_rho = logp.gather(-1, a).squeeze(-1) - lmu.gather(-1, a).squeeze(-1)
        ratio = torch.exp(log_rho)
        rho = torch.clamp(ratio, max=hp["rho_bar"])
        c = hp["lambda_"] * torch.clamp(ratio, max=hp["c_bar"])
        pgr = torch.clamp(ratio, max=hp["pg_rho_bar"])
        v = values.detach()
        delta = rho * (rewards + discounts * v[1:] - v[:-1])
        acc = torch.zeros_like(v[0])
        accs = [None] * T
        for t in range(T - 1, -1, -1):
            acc = delta[t] + discounts[t] * c[t] * acc
            accs[t] = acc
        vs = v[:-1] + torch.stack(accs)
        vs_next = torch.cat([vs[1:], v[-1:]], 0)
        pg_adv = pgr * (rewards + discounts * vs_next - v[:-1])
    lpa = logp.gather(-1, actions.long().unsqueeze(-1)).squeeze(-1)
    pg = -(pg_adv * lpa).sum()
    base = 0.5 * ((vs - values[:-1]) ** 2).sum()
    ent = (torch.exp(logp) * logp).sum()
    return pg + hp["baseline_cost"] * base + hp["entropy_cost"] * ent, (pg, base, ent)


class TorchLearner:
    """One learner step on CPU tensors; parameters/moments as flat fp32 tensors."""

    def __init__(self, arch, params: np.ndarray, A=18, D=128, H=256, lr=5e-4, b1=0.9,
                 b2=0.999, eps=1e-8, max_grad_norm=40.0):
        self.arch, self.A, self.D, self.H = arch, A, D, H
        self.p = torch.tensor(np.asarray(params, np.float32))
        self.m = torch.zeros_like(self.p)
        self.v = torch.zeros_like(self.p)
        self.lr, self.b1, self.b2, self.eps, self.clip = lr, b1, b2, eps, max_grad_norm
        self.t = 0

    def grads(self, batch):
        """batch: dict of numpy arrays (oracle.synth_batch layout). Returns (grad, losses)."""
        p = self.p.detach().requires_grad_(True)
        T, B = batch["actions"].shape
        A = self.A
        if self.arch == "mlp":
            out = mlp_forward(p, torch.from_numpy(batch["obs"]).reshape(-1, self.D), self.D, self.H, A)
        else:
            fr = torch.from_numpy(batch["frames"]).reshape(-1, 84, 84, 4)
            out = atari_forward(p, fr, A)
        logits = out[:, :A].reshape(T + 1, B, A)
        values = out[:, A].reshape(T + 1, B)
        total, parts = vtrace_loss(logits[:T], torch.from_numpy(batch["mu"]),
                                   torch.from_numpy(batch["actions"]),
                                   torch.from_numpy(batch["rewards"]),
                                   torch.from_numpy(batch["discounts"]), values)
        (g,) = torch.autograd.grad(total, p)
        return g, [float(x.detach()) for x in parts]

    def step(self, batch):
        g, losses = self.grads(batch)
        with torch.no_grad():
            norm = float(torch.linalg.vector_norm(g.double()))
            if self.clip > 0 and norm > self.clip:
                g = g * (self.clip / (norm + 1e-6))
            self.t += 1
            self.m.mul_(self.b1).add_(g, alpha=1 - self.b1)
            self.v.mul_(self.b2).addcmul_(g, g, value=1 - self.b2)
            mh = self.m / (1 - self.b1 ** self.t)
            vh = self.v / (1 - self.b2 ** self.t)
            self.p.sub_(self.lr * mh / (vh.sqrt() + self.eps))
        return losses, norm
