"""TEST INFRASTRUCTURE / CPU BASELINE ONLY -- never imported by the product path.

The reference's FarmerLstm train step (scripts/gpu_benchmark.py:11-44, 99-125) on PyTorch's
CPU kernels, driven from the same fp32 parameter blob as the device path (state_dict order,
oracle/farmer_oracle.py), so scripts/farmer_bench.py can time the reference's own CPU
execution stack (torch CPU: oneDNN LSTM / MKL GEMMs, autograd, torch.optim) on the GPU box's
host cores, where /root/reference itself is not available. Gradient-equal to the numpy oracle
(tests/test_farmer_oracle.py covers the oracle; tests/test_torch_baseline.py this port).
"""
from __future__ import annotations

import numpy as np
import torch

from . import farmer_oracle as fo


class TorchFarmer:
    def __init__(self, params: np.ndarray, loss="mse", optimizer="adam", lr=1e-3):
        self.lstm = torch.nn.LSTM(fo.I_IN, fo.HID, batch_first=True)
        dims = [(fo.HID + fo.X_IN, fo.DW)] + [(fo.DW, fo.DW)] * 4 + [(fo.DW, 1)]
        self.dense = torch.nn.ModuleList([torch.nn.Linear(i, o) for i, o in dims])
        self.params = list(self.lstm.parameters()) + list(self.dense.parameters())
        with torch.no_grad():
            for prm, (n, (a, b, s)) in zip(self.params, fo.offsets().items()):
                assert tuple(prm.shape) == tuple(s), (n, prm.shape, s)
                prm.copy_(torch.from_numpy(np.ascontiguousarray(params[a:b]).reshape(s)))
        self.crit = {"mse": torch.nn.MSELoss(), "mae": torch.nn.L1Loss(), "huber": torch.nn.SmoothL1Loss()}[loss]
        self.opt = {"adam": torch.optim.Adam, "sgd": torch.optim.SGD, "adamw": torch.optim.AdamW}[optimizer](
            self.params, lr=lr)

    def forward(self, z, x):
        out, _ = self.lstm(z)
        h = torch.cat([out[:, -1, :], x], dim=-1)
        for i, lin in enumerate(self.dense):
            h = lin(h)
            if i < len(self.dense) - 1:
                h = torch.relu(h)
        return h

    def step(self, z, x, y) -> float:
        self.opt.zero_grad()
        loss = self.crit(self.forward(z, x), y)
        loss.backward()
        self.opt.step()
        return float(loss.item())

    def grads(self) -> np.ndarray:
        return np.concatenate([p.grad.detach().numpy().reshape(-1) for p in self.params])
