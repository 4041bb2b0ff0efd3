"""Oracle (C restatement) pinned against the golden fixtures and hand-derived KATs.

The reference has no vectors for this path ("parity unpinned by the
reference"); the fixtures come from an independent torch-autograd restatement
(tests/golden/make_golden.py) and the KATs below are derived by hand from IMPALA eq. 1.
"""
import glob
import math
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(__file__), "golden")
HP_KEYS = ["rho_bar", "c_bar", "pg_rho_bar", "lambda_", "baseline_cost", "entropy_cost"]


def _close(a, b, tol=1e-5):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    err = np.abs(a - b) / np.maximum(1.0, np.abs(b))
    assert err.max() <= tol, f"max rel err {err.max():.3e}"


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "vtrace_*.npz"))))
def test_vtrace_oracle_vs_golden(orc, path):
    z = np.load(path)
    hp = dict(zip(HP_KEYS, z["hp"].tolist()))
    out = orc.vtrace_loss(z["pi"], z["mu"], z["actions"], z["rewards"], z["discounts"],
                          z["values"], **hp)
    for k in ("vs", "pg_adv", "dlogits", "dvalue"):
        _close(out[k], z[k])
    np.testing.assert_allclose(out["losses"], z["losses"], rtol=1e-9, atol=1e-9)


def test_vtrace_kat_on_policy_T2(orc):
    """Hand-derived: T=2, B=1, A=2, pi == mu (rho = c = 1), uniform logits.
    V = [1, 2], bootstrap 3, r = [1, 0], gamma = 0.5.
    delta_1 = 0 + 0.5*3 - 2 = -0.5 ; acc_1 = -0.5 ; vs_1 = 1.5
    delta_0 = 1 + 0.5*2 - 1 = 1 ; acc_0 = 1 + 0.5*(-0.5) = 0.75 ; vs_0 = 1.75
    pg_adv_1 = 0 + 0.5*3 - 2 = -0.5 ; pg_adv_0 = 1 + 0.5*1.5 - 1 = 0.75
    """
    z = np.zeros((2, 1, 2), np.float32)
    out = orc.vtrace_loss(z, z, np.array([[0], [1]]), np.array([[1.0], [0.0]]),
                          np.array([[0.5], [0.5]]), np.array([[1.0], [2.0], [3.0]]),
                          entropy_cost=0.0, baseline_cost=1.0)
    np.testing.assert_allclose(out["vs"][:, 0], [1.75, 1.5], rtol=0, atol=1e-7)
    np.testing.assert_allclose(out["pg_adv"][:, 0], [0.75, -0.5], rtol=0, atol=1e-7)
    # dvalue = bc*(V - vs); bootstrap row 0
    np.testing.assert_allclose(out["dvalue"][:, 0], [-0.75, 0.5, 0.0], atol=1e-7)
    # dlogits = -adv*(onehot - 0.5)
    np.testing.assert_allclose(out["dlogits"][0, 0], [-0.375, 0.375], atol=1e-7)
    np.testing.assert_allclose(out["dlogits"][1, 0], [-0.25, 0.25], atol=1e-7)
    ln2 = math.log(2.0)
    np.testing.assert_allclose(out["losses"],
                               [0.75 * ln2 - 0.5 * ln2, 0.5 * (0.75 ** 2 + 0.5 ** 2), -2 * ln2],
                               rtol=1e-12)


def test_vtrace_kat_clipping(orc):
    """T=1: pi puts all mass on the taken action relative to mu -> rho clipped to rho_bar."""
    pi = np.array([[[10.0, -10.0]]], np.float32)
    mu = np.array([[[0.0, 0.0]]], np.float32)
    out = orc.vtrace_loss(pi, mu, np.array([[0]]), np.array([[1.0]]), np.array([[0.9]]),
                          np.array([[0.0], [1.0]]), rho_bar=0.7, pg_rho_bar=0.3)
    # ratio ~ 2 -> rho = 0.7 ; vs = 0 + 0.7*(1 + 0.9*1 - 0) = 1.33 ; pg_adv = 0.3*(1.9)
    np.testing.assert_allclose(out["vs"][0, 0], 1.33, rtol=1e-6)
    np.testing.assert_allclose(out["pg_adv"][0, 0], 0.57, rtol=1e-6)


@pytest.mark.parametrize("name", ["small", "full"])
def test_mlp_oracle_vs_golden(orc, name):
    from tests.golden.make_golden import mlp_params
    z = np.load(os.path.join(GOLD, f"mlp_{name}.npz"))
    N, D, H, A = z["dims"].tolist()
    p = mlp_params(int(z["seed"]), D, H, A)
    h1, h2, out = orc.mlp_forward(z["obs"], p, H=H, A=A)
    _close(out, z["out"], 1e-5)
    g = orc.mlp_backward(z["obs"], p, h1, h2, z["dout"], H=H, A=A)
    _close(g, z["grads"], 1e-5)


def test_atari_oracle_vs_golden(orc):
    from tests.golden.make_golden import atari_params, ATARI_FC_STRIDE
    z = np.load(os.path.join(GOLD, "atari_n2.npz"))
    N, A = z["dims"].tolist()
    p = atari_params(int(z["seed"]), A)
    rs = np.random.RandomState(int(z["seed"]) + 2000)
    frames = rs.randint(0, 256, size=(N, 84, 84, 4)).astype(np.uint8)
    acts = orc.atari_forward(frames, p, A=A, bf16_emul=False)
    _close(acts["out"], z["out"], 1e-5)
    _close(acts["h"], z["h"], 1e-5)
    g = orc.atari_backward(frames, p, acts, z["dout"], A=A, bf16_emul=False)
    sizes = [8192, 32, 32768, 64, 36864, 64, 3136 * 512, 512, 512 * (A + 1), A + 1]
    off = np.cumsum([0] + sizes)
    kept = np.concatenate([g[off[0]:off[6]], g[off[6]:off[7]][::ATARI_FC_STRIDE], g[off[7]:]])
    scale = np.abs(z["grads_kept"]).max()
    np.testing.assert_allclose(kept / scale, z["grads_kept"] / scale, atol=2e-6)


def test_adam_matches_closed_form(orc):
    p = np.array([1.0, -2.0], np.float32)
    g = np.array([0.5, -0.25], np.float32)
    m = np.zeros(2, np.float32)
    v = np.zeros(2, np.float32)
    orc.adam(p, g, m, v, 1e-3, 0.9, 0.999, 1e-8, 1)
    # step 1: mhat = g, vhat = g^2 -> p -= lr * sign(g)
    np.testing.assert_allclose(p, [1.0 - 1e-3, -2.0 + 1e-3], rtol=1e-6)


def test_clip_grad_norm(orc):
    g = np.array([3.0, 4.0], np.float32)
    n = orc.clip_grad_norm(g, 1.0)
    assert abs(n - 5.0) < 1e-9
    np.testing.assert_allclose(np.linalg.norm(g), 1.0, rtol=1e-5)


def test_philox_known_answer(orc):
    # Philox4x32-10 KAT (Salmon et al. 2011, Random123 kat_vectors): ctr=0, key=0
    np.testing.assert_array_equal(orc.philox4(0, 0, 0),
                                  np.array([0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8],
                                           np.uint32))


def test_synth_shard_independent_of_gpu_count(orc):
    full = orc.synth_batch(42, T=4, B=8, A=18, D=16)
    sh = orc.synth_batch(42, T=4, B=4, A=18, D=16, B_glob=8, b_off=4)
    for k in ("obs", "mu", "actions", "rewards", "discounts"):
        np.testing.assert_array_equal(full[k][:, 4:8], sh[k])
    assert full["actions"].min() >= 0 and full["actions"].max() < 18
    assert set(np.unique(full["rewards"]).tolist()) <= {-1.0, 0.0, 1.0}
    o = orc.synth_batch(7, T=63, B=64, A=18, D=32)["obs"]
    assert abs(o.mean()) < 0.02 and abs(o.std() - 1.0) < 0.02


def _bf16_bits(a, rs=None):
    return (np.asarray(a, np.float32).view(np.uint32) >> 16).astype(np.uint16)


def test_conv_wgrad_f64_checker_matches_direct_sums(orc):
    """The full-depth gradient test's fp64 checker (orc_conv_wgrad_f64) against direct numpy sums:
    conv1 on u8 frames, conv2 on a1 in NHWC and in conv21's parity-plane order."""
    rs = np.random.RandomState(4)
    N = 5
    fr = rs.randint(0, 256, (N, 84, 84, 4)).astype(np.uint8)
    d1 = _bf16_bits(rs.randn(N, 20, 20, 32))
    cos = [0, 9, 31]
    got = orc.conv_wgrad_f64(fr, d1, N, 84, 4, 8, 4, 32, cos, x_kind=0)
    df = (d1.astype(np.uint32) << 16).view(np.float32).astype(np.float64)[..., cos]
    for ky, kx in [(0, 0), (3, 7), (7, 7)]:
        ref = np.einsum("nyxc,nyxo->co", fr[:, ky:ky + 77:4, kx:kx + 77:4].astype(np.float64), df)
        np.testing.assert_allclose(got[ky, kx], ref, rtol=1e-12)
    a1 = _bf16_bits(rs.randn(N, 20, 20, 32))
    d2 = _bf16_bits(rs.randn(N, 9, 9, 64))
    planar = a1.reshape(N, 10, 2, 10, 2, 32).transpose(0, 2, 4, 1, 3, 5).copy()  # [iy&1][ix&1][iy>>1][ix>>1]
    c2 = [1, 63]
    g_nhwc = orc.conv_wgrad_f64(a1, d2, N, 20, 32, 4, 2, 64, c2, x_kind=1)
    g_plan = orc.conv_wgrad_f64(planar, d2, N, 20, 32, 4, 2, 64, c2, x_kind=2)
    np.testing.assert_array_equal(g_nhwc, g_plan)
    af = (a1.astype(np.uint32) << 16).view(np.float32).astype(np.float64)
    d2f = (d2.astype(np.uint32) << 16).view(np.float32).astype(np.float64)[..., c2]
    for ky in range(4):
        for kx in range(4):
            ref = np.einsum("nyxc,nyxo->co", af[:, ky:ky + 17:2, kx:kx + 17:2], d2f)
            np.testing.assert_allclose(g_nhwc[ky, kx], ref, rtol=1e-12)
