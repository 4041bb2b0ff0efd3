"""Diagnostic: repeat the fused conv2/conv1 backward at small sizes and report non-finite
gradient entries (which parameter block, which rows), and the max deviation between
repeated identical steps."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from freeimpala_amd.learner import DeviceLearner  # noqa: E402

names = ["c1W", "c1b", "c2W", "c2b", "c3W", "c3b", "fcW", "fcb", "hW", "hb"]
sizes = [8192, 32, 32768, 64, 36864, 64, 3136 * 512, 512, 512 * 19, 19]
off = np.cumsum([0] + sizes)
for T, B in [(2, 16), (3, 32), (5, 176)]:
    ref = None
    for rep in range(4):
        L = DeviceLearner("atari", seq_len=T, batch=B, num_actions=18, optimizer="sgd", lr=1e-3,
                          max_grad_norm=0.0, seed=3)
        L.synth(seed=T * 100 + B)
        L.step_resident()
        g = L.tensor("grads")
        L.close()
        bad = {}
        for i, nm in enumerate(names):
            blk = g[off[i]:off[i + 1]]
            nb = np.flatnonzero(~np.isfinite(blk))
            if nb.size:
                bad[nm] = (nb.size, nb[:8].tolist())
        dev = None
        if ref is not None:
            dev = {nm: float(np.nanmax(np.abs(g[off[i]:off[i + 1]] - ref[off[i]:off[i + 1]])))
                   for i, nm in enumerate(names[:4])}
        else:
            ref = g
        print(f"T={T} B={B} rep={rep} nonfinite={bad} dev_vs_rep0={dev}", flush=True)
