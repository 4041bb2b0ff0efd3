"""TEST INFRASTRUCTURE ONLY -- never imported by the product path.

CPU restatement (numpy, float64 accumulation) of the reference's only neural network and its
training step: FarmerLstmModel + criterion + optimizer step, as defined in
  /root/reference/scripts/gpu_benchmark.py:11-44   (model: LSTM(162->128, batch_first), last
                                                    timestep, cat with x[484], 5 x (Linear 512 +
                                                    ReLU), Linear(512 -> 1))
  /root/reference/scripts/gpu_benchmark.py:46-66   (criterion mse / mae / huber = MSELoss,
                                                    L1Loss, SmoothL1Loss; optimizer adam / sgd /
                                                    adamw with torch defaults)
  /root/reference/scripts/gpu_benchmark.py:99-125  (train step: zero_grad, forward, loss,
                                                    backward, optimizer.step)
  /root/reference/cmd/libtorch_bench/main.cpp:14-42, 117-135 (the same model / step in libtorch)
Pinned against tests/golden/farmer_*.npz, which tests/golden/make_farmer_golden.py generates by
running the reference's own FarmerLstmModel (imported from gpu_benchmark.py) on these
parameters and inputs (tests/test_farmer_oracle.py).

Parameter blob = the model's state_dict order, PyTorch layouts ([out][in] weights), fp32:
  lstm.weight_ih_l0 [512][162]  lstm.weight_hh_l0 [512][128]  lstm.bias_ih_l0 [512]
  lstm.bias_hh_l0 [512]  dense1.weight [512][612] dense1.bias [512]  dense2..5 [512][512] + [512]
  dense6.weight [1][512] dense6.bias [1]          (1,514,497 floats; LSTM gate order i, f, g, o)
"""
from __future__ import annotations

import numpy as np

I_IN, HID, X_IN, DW = 162, 128, 484, 512
G4 = 4 * HID

SHAPES = [("lstm.weight_ih_l0", (G4, I_IN)), ("lstm.weight_hh_l0", (G4, HID)),
          ("lstm.bias_ih_l0", (G4,)), ("lstm.bias_hh_l0", (G4,)),
          ("dense1.weight", (DW, HID + X_IN)), ("dense1.bias", (DW,))]
for _i in range(2, 6):
    SHAPES += [(f"dense{_i}.weight", (DW, DW)), (f"dense{_i}.bias", (DW,))]
SHAPES += [("dense6.weight", (1, DW)), ("dense6.bias", (1,))]
PARAM_COUNT = sum(int(np.prod(s)) for _, s in SHAPES)  # 1,514,497 (gpu_benchmark's model)

LOSSES = {"mse": 0, "mae": 1, "huber": 2}
OPTIMIZERS = {"adam": 0, "sgd": 1, "adamw": 2}


def offsets():
    out, o = {}, 0
    for n, s in SHAPES:
        k = int(np.prod(s))
        out[n] = (o, o + k, s)
        o += k
    return out


def views(p):
    return {n: p[a:b].reshape(s) for n, (a, b, s) in offsets().items()}


def gen_params(seed):
    """Deterministic parameters (uniform +-1/sqrt(fan_in), torch's default init scale)."""
    rs = np.random.RandomState(seed)
    parts = []
    for n, s in SHAPES:
        fan = HID if n.startswith("lstm") else (s[1] if len(s) == 2 else None)
        if fan is None:  # a dense bias: fan_in of its layer
            fan = HID + X_IN if n == "dense1.bias" else DW
        k = 1.0 / np.sqrt(fan)
        parts.append(rs.uniform(-k, k, int(np.prod(s))).astype(np.float32))
    return np.concatenate(parts)


def gen_inputs(seed, B, T):
    rs = np.random.RandomState(seed)
    z = rs.standard_normal((B, T, I_IN)).astype(np.float32)
    x = rs.standard_normal((B, X_IN)).astype(np.float32)
    y = rs.standard_normal((B, 1)).astype(np.float32)
    return z, x, y


def _sig(a):
    return 1.0 / (1.0 + np.exp(-a))


def forward(p, z, x):
    """Returns value [B,1] and the saved activations for backward (float64)."""
    v = {k: a.astype(np.float64) for k, a in views(p).items()}
    B, T, _ = z.shape
    z = z.astype(np.float64)
    h = np.zeros((B, HID))
    c = np.zeros((B, HID))
    gates, cs, hs = [], [], []
    for t in range(T):
        a = z[:, t] @ v["lstm.weight_ih_l0"].T + v["lstm.bias_ih_l0"] + h @ v["lstm.weight_hh_l0"].T \
            + v["lstm.bias_hh_l0"]
        i, f, g, o = _sig(a[:, :HID]), _sig(a[:, HID:2 * HID]), np.tanh(a[:, 2 * HID:3 * HID]), _sig(a[:, 3 * HID:])
        hs.append(h)
        c = f * c + i * g
        h = o * np.tanh(c)
        gates.append((i, f, g, o))
        cs.append(c)
    acts = [np.concatenate([h, x.astype(np.float64)], axis=1)]
    for l in range(1, 6):
        acts.append(np.maximum(acts[-1] @ v[f"dense{l}.weight"].T + v[f"dense{l}.bias"], 0.0))
    val = acts[-1] @ v["dense6.weight"].T + v["dense6.bias"]
    return val, dict(gates=gates, cs=cs, hprev=hs, acts=acts, z=z)


def loss_and_grad(val, y, loss="mse"):
    d = val - y.astype(np.float64)
    n = d.size
    if loss == "mse":
        return float(np.mean(d * d)), 2.0 * d / n
    if loss == "mae":
        return float(np.mean(np.abs(d))), np.sign(d) / n
    ad = np.abs(d)  # SmoothL1Loss, beta = 1
    return float(np.mean(np.where(ad < 1.0, 0.5 * d * d, ad - 0.5))), np.where(ad < 1.0, d, np.sign(d)) / n


def backward(p, saved, dval):
    v = {k: a.astype(np.float64) for k, a in views(p).items()}
    g = {}
    acts = saved["acts"]
    g["dense6.weight"] = dval.T @ acts[5]
    g["dense6.bias"] = dval.sum(0)
    da = (dval @ v["dense6.weight"]) * (acts[5] > 0)
    for l in range(5, 0, -1):
        g[f"dense{l}.weight"] = da.T @ acts[l - 1]
        g[f"dense{l}.bias"] = da.sum(0)
        da = da @ v[f"dense{l}.weight"]
        if l > 1:
            da = da * (acts[l - 1] > 0)
    dh = da[:, :HID]
    z = saved["z"]
    B, T, _ = z.shape
    dc = np.zeros((B, HID))
    gWih = np.zeros((G4, I_IN))
    gWhh = np.zeros((G4, HID))
    gb = np.zeros(G4)
    for t in range(T - 1, -1, -1):
        i, f, gg, o = saved["gates"][t]
        c = saved["cs"][t]
        cprev = saved["cs"][t - 1] if t > 0 else np.zeros_like(c)
        tc = np.tanh(c)
        do = dh * tc
        dc = dc + dh * o * (1.0 - tc * tc)
        di, dg, df = dc * gg, dc * i, dc * cprev
        da4 = np.concatenate([di * i * (1 - i), df * f * (1 - f), dg * (1 - gg * gg), do * o * (1 - o)], axis=1)
        gWih += da4.T @ z[:, t]
        gWhh += da4.T @ saved["hprev"][t]
        gb += da4.sum(0)
        dh = da4 @ v["lstm.weight_hh_l0"]
        dc = dc * f
    g["lstm.weight_ih_l0"] = gWih
    g["lstm.weight_hh_l0"] = gWhh
    g["lstm.bias_ih_l0"] = gb
    g["lstm.bias_hh_l0"] = gb.copy()
    return np.concatenate([g[n].reshape(-1) for n, _ in SHAPES])


class Optimizer:
    """torch.optim.{Adam, SGD, AdamW} with torch's defaults (betas 0.9/0.999, eps 1e-8,
    AdamW weight_decay 0.01), in float64."""

    def __init__(self, kind, lr, n, weight_decay=None):
        self.kind, self.lr, self.t = kind, lr, 0
        self.wd = (0.01 if kind == "adamw" else 0.0) if weight_decay is None else weight_decay
        self.m = np.zeros(n)
        self.v = np.zeros(n)

    def step(self, p, g):
        p = p.astype(np.float64)
        if self.kind == "sgd":
            return p - self.lr * g
        self.t += 1
        b1, b2, eps = 0.9, 0.999, 1e-8
        if self.kind == "adamw":
            p = p * (1.0 - self.lr * self.wd)
        self.m = b1 * self.m + (1 - b1) * g
        self.v = b2 * self.v + (1 - b2) * g * g
        mh = self.m / (1 - b1 ** self.t)
        vh = self.v / (1 - b2 ** self.t)
        return p - self.lr * mh / (np.sqrt(vh) + eps)


def train_step(p, opt, z, x, y, loss="mse"):
    """One reference train step: returns (value, loss, grads, new params float32)."""
    val, saved = forward(p, z, x)
    lv, dval = loss_and_grad(val, y, loss)
    g = backward(p, saved, dval)
    return val, lv, g, opt.step(p, g).astype(np.float32)
