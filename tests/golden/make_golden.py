"""Generate the golden fixtures under tests/golden/ with an INDEPENDENT restatement.

The reference (filevich/freeimpala) has no V-trace, loss or network (SURVEY.md section 0,
learner.h:32-49), hence no golden vectors. These fixtures pin the C oracle against a
second, independent restatement written directly in PyTorch (float64, autograd for every
gradient -- the oracle's gradients are analytic), following the IMPALA spec
(arXiv:1802.01561 eq. 1, section 4.2) and the torchbeast/scalable_agent
``from_importance_weights`` formulation.

Run in this container (torch CPU):  python tests/golden/make_golden.py
Only inputs/outputs are committed (.npz, no pickles); torch never ships to the GPU box.
Parameters of the network cases are regenerated from numpy.random.RandomState(seed) by the
tests, so the fixtures stay small.
"""
from __future__ import annotations

import os

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
torch.set_default_dtype(torch.float64)


# --------------------------------------------------------------------------- V-trace
def vtrace_torch(pi, mu, actions, rewards, discounts, values, rho_bar=1.0, c_bar=1.0,
                 pg_rho_bar=1.0, lambda_=1.0, baseline_cost=0.5, entropy_cost=0.01):
    """Independent restatement: log-rhos via log_softmax gather, python-loop reverse scan,
    losses as sums; gradients by autograd."""
    pi = torch.tensor(pi, dtype=torch.float64, requires_grad=True)
    values_t = torch.tensor(values, dtype=torch.float64, requires_grad=True)
    mu = torch.tensor(mu, dtype=torch.float64)
    act = torch.tensor(actions, dtype=torch.int64)
    r = torch.tensor(rewards, dtype=torch.float64)
    disc = torch.tensor(discounts, dtype=torch.float64)
    T = pi.shape[0]
    logp_pi = F.log_softmax(pi, dim=-1)
    logp_mu = F.log_softmax(mu, dim=-1)
    lp_a = logp_pi.gather(-1, act.unsqueeze(-1)).squeeze(-1)
    lm_a = logp_mu.gather(-1, act.unsqueeze(-1)).squeeze(-1)
    with torch.no_grad():
        log_rhos = lp_a - lm_a
        rhos = torch.exp(log_rhos)
        clipped_rhos = torch.clamp(rhos, max=rho_bar)
        cs = lambda_ * torch.clamp(rhos, max=c_bar)
        V = values_t[:T]
        boot = values_t[T]
        v_tp1 = torch.cat([V[1:], boot.unsqueeze(0)], 0)
        deltas = clipped_rhos * (r + disc * v_tp1 - V)
        acc = torch.zeros_like(boot)
        res = []
        for t in reversed(range(T)):
            acc = deltas[t] + disc[t] * cs[t] * acc
            res.append(acc)
        vs_minus_v = torch.stack(list(reversed(res)), 0)
        vs = vs_minus_v + V
        vs_tp1 = torch.cat([vs[1:], boot.unsqueeze(0)], 0)
        pg_adv = torch.clamp(rhos, max=pg_rho_bar) * (r + disc * vs_tp1 - V)
    pg_loss = torch.sum(-lp_a * pg_adv)
    base_loss = 0.5 * torch.sum((vs - values_t[:T]) ** 2)
    ent_loss = torch.sum(torch.exp(logp_pi) * logp_pi)
    total = pg_loss + baseline_cost * base_loss + entropy_cost * ent_loss
    total.backward()
    return dict(vs=vs.numpy(), pg_adv=pg_adv.numpy(), dlogits=pi.grad.numpy(),
                dvalue=values_t.grad.numpy(),
                losses=np.array([pg_loss.item(), base_loss.item(), ent_loss.item()]))


def vtrace_case(name, seed, T, B, A, logit_scale=1.0, done_p=0.1, gamma=0.99, **hp):
    rs = np.random.RandomState(seed)
    pi = (rs.randn(T, B, A) * logit_scale).astype(np.float32)
    mu = (rs.randn(T, B, A) * logit_scale).astype(np.float32)
    actions = rs.randint(0, A, size=(T, B)).astype(np.int32)
    rewards = rs.choice([-1.0, 0.0, 1.0], size=(T, B)).astype(np.float32)
    done = rs.rand(T, B) < done_p
    discounts = np.where(done, 0.0, gamma).astype(np.float32)
    values = rs.randn(T + 1, B).astype(np.float32)
    out = vtrace_torch(pi, mu, actions, rewards, discounts, values, **hp)
    hp_arr = np.array([hp.get("rho_bar", 1.0), hp.get("c_bar", 1.0), hp.get("pg_rho_bar", 1.0),
                       hp.get("lambda_", 1.0), hp.get("baseline_cost", 0.5),
                       hp.get("entropy_cost", 0.01)], np.float64)
    np.savez_compressed(os.path.join(HERE, f"vtrace_{name}.npz"), pi=pi, mu=mu, actions=actions,
                        rewards=rewards, discounts=discounts, values=values, hp=hp_arr,
                        **{k: np.asarray(v, np.float64) for k, v in out.items()})


# --------------------------------------------------------------------------- MLP
def mlp_params(seed, D, H, A):
    rs = np.random.RandomState(seed)
    O = A + 1
    shapes = [(D, H), (H,), (H, H), (H,), (H, O), (O,)]
    return np.concatenate([(rs.randn(*s) * 0.2).astype(np.float32).ravel() for s in shapes])


def mlp_case(name, seed, N, D, H, A):
    rs = np.random.RandomState(seed + 1000)
    obs = rs.randn(N, D).astype(np.float32)
    dout = rs.randn(N, A + 1).astype(np.float32)
    p = torch.tensor(mlp_params(seed, D, H, A), dtype=torch.float64, requires_grad=True)
    O = A + 1
    sizes = [D * H, H, H * H, H, H * O, O]
    W1, b1, W2, b2, Wh, bh = torch.split(p, sizes)
    x = torch.tensor(obs, dtype=torch.float64)
    h1 = torch.relu(x @ W1.view(D, H) + b1)
    h2 = torch.relu(h1 @ W2.view(H, H) + b2)
    out = h2 @ Wh.view(H, O) + bh
    (out * torch.tensor(dout, dtype=torch.float64)).sum().backward()
    np.savez_compressed(os.path.join(HERE, f"mlp_{name}.npz"), seed=seed, dims=np.array([N, D, H, A]),
                        obs=obs, dout=dout, out=out.detach().numpy(), h2=h2.detach().numpy(),
                        grads=p.grad.numpy())


# --------------------------------------------------------------------------- Atari net
def atari_params(seed, A):
    rs = np.random.RandomState(seed)
    O = A + 1
    shapes = [(8, 8, 4, 32), (32,), (4, 4, 32, 64), (64,), (3, 3, 64, 64), (64,),
              (3136, 512), (512,), (512, O), (O,)]
    fan = [256, 1, 512, 1, 576, 1, 3136, 1, 512, 1]
    return np.concatenate([(rs.randn(*s) / np.sqrt(f) * (1.0 if len(s) > 1 else 0.1))
                           .astype(np.float32).ravel() for s, f in zip(shapes, fan)])


ATARI_FC_STRIDE = 97  # fc weight grads are stored subsampled (every 97th element)


def atari_case(name, seed, N, A):
    rs = np.random.RandomState(seed + 2000)
    frames = rs.randint(0, 256, size=(N, 84, 84, 4)).astype(np.uint8)
    dout = rs.randn(N, A + 1).astype(np.float32)
    O = A + 1
    p = torch.tensor(atari_params(seed, A), dtype=torch.float64, requires_grad=True)
    sizes = [8192, 32, 32768, 64, 36864, 64, 3136 * 512, 512, 512 * O, O]
    c1w, c1b, c2w, c2b, c3w, c3b, fw, fb, hw, hb = torch.split(p, sizes)
    x = torch.tensor(frames, dtype=torch.float64).permute(0, 3, 1, 2) / 255.0
    y = torch.relu(F.conv2d(x, c1w.view(8, 8, 4, 32).permute(3, 2, 0, 1), c1b, stride=4))
    y = torch.relu(F.conv2d(y, c2w.view(4, 4, 32, 64).permute(3, 2, 0, 1), c2b, stride=2))
    y = torch.relu(F.conv2d(y, c3w.view(3, 3, 64, 64).permute(3, 2, 0, 1), c3b, stride=1))
    y = y.permute(0, 2, 3, 1).reshape(N, 3136)
    h = torch.relu(y @ fw.view(3136, 512) + fb)
    out = h @ hw.view(512, O) + hb
    (out * torch.tensor(dout, dtype=torch.float64)).sum().backward()
    g = p.grad.numpy()
    off = np.cumsum([0] + sizes)
    keep = np.concatenate([g[off[0]:off[6]], g[off[6]:off[7]][::ATARI_FC_STRIDE], g[off[7]:]])
    np.savez_compressed(os.path.join(HERE, f"atari_{name}.npz"), seed=seed, dims=np.array([N, A]),
                        dout=dout, out=out.detach().numpy(), h=h.detach().numpy(), grads_kept=keep,
                        fc_stride=ATARI_FC_STRIDE)


def main():
    vtrace_case("small", 1, T=5, B=3, A=4)
    vtrace_case("t1_gamma0", 2, T=1, B=8, A=2, gamma=0.0)
    vtrace_case("adversarial", 3, T=100, B=8, A=18, logit_scale=12.0, done_p=0.05,
                rho_bar=0.8, c_bar=0.6, pg_rho_bar=1.5, lambda_=0.95,
                baseline_cost=0.25, entropy_cost=0.02)
    vtrace_case("config2_slice", 4, T=100, B=16, A=18)
    vtrace_case("alldone", 5, T=7, B=5, A=6, done_p=1.0)
    mlp_case("small", 11, N=6, D=16, H=32, A=4)
    mlp_case("full", 12, N=4, D=128, H=256, A=18)
    atari_case("n2", 21, N=2, A=18)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
