"""Helpers for the FarmerLstm golden fixtures (tests/golden/farmer_*.npz, made from the
reference's own model by tests/golden/make_farmer_golden.py)."""
import glob
import os

import numpy as np

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def cases():
    return sorted(glob.glob(os.path.join(GOLD, "farmer_*.npz")))


def load(path):
    z = np.load(path)
    return {k: z[k] for k in z.files}


def _ref_grad(g, step, n):
    key = f"step{step}/grad/{n}"
    return g[key] if key in g else g[key + ":val"]


def well_conditioned(g, step, n, rel=1e-3):
    """Adam / AdamW normalise every element's step by its own gradient magnitude: where the
    gradient is ~0 (saturated gates, ~1e-9 in fp32) any rounding of it changes the update by up
    to lr. Positions whose reference gradient stayed above rel * max|grad| of the tensor in
    every step so far are the ones an Adam parameter comparison can pin."""
    ok = None
    for s in range(step + 1):
        a = np.abs(_ref_grad(g, s, n).astype(np.float64))
        m = a >= rel * max(a.max(), 1e-30)
        ok = m if ok is None else ok & m
    return ok


def compare_blob(g, step, kind, blob, names_offsets, rtol, atol_frac, what="", adam=False):
    """blob: the full flat array (grads or params) in state_dict order. Full tensors are
    compared elementwise (|d| <= atol_frac * max|ref| + rtol |ref|); sampled ones at their
    indices plus the tensor sum / sum of squares (relative). adam=True (parameters after an
    Adam-family step): only well-conditioned positions elementwise, sums at a looser bar."""
    worst = 0.0
    for n, (a, b, s) in names_offsets.items():
        t = np.asarray(blob[a:b], np.float64)
        key = f"step{step}/{kind}/{n}"
        if key in g:
            ref = g[key].astype(np.float64)
            got = t
        else:
            idx = g[key + ":idx"]
            ref = g[key + ":val"].astype(np.float64)
            got = t[idx]
            for agg, val in (("sum", t.sum()), ("sumsq", (t * t).sum())):
                r = float(g[f"{key}:{agg}"])
                scale = float(g[f"{key}:sumsq"]) ** 0.5 * np.sqrt(t.size) if agg == "sum" else abs(r)
                err = abs(val - r) / max(scale, 1e-30)
                bar = max(rtol, atol_frac) * (1e3 if adam else 10)
                assert err <= bar, f"{what} {key}:{agg} {val} vs {r} (err {err:.2e})"
        scale = max(1e-30, np.abs(ref).max())
        if adam:
            m = well_conditioned(g, step, n)
            got, ref = got[m], ref[m]
        err = np.abs(got - ref) - rtol * np.abs(ref)
        e = float(err.max()) / scale
        worst = max(worst, e)
        assert e <= atol_frac, f"{what} {key}: err {e:.2e} (max|ref| {scale:.3e})"
    return worst
