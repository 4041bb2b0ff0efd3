"""GPU parity of the FarmerLstm train step (farmer.hip through include/fi_farmer.h).

Pinned by the REFERENCE: tests/golden/farmer_*.npz hold the values, loss, gradients and updated
parameters of the reference's own gpu_benchmark.FarmerLstmModel train step (adam / adamw /
sgd x mse / huber / mae, two steps each), generated in the build container by
tests/golden/make_farmer_golden.py. Larger shapes (T = 100, ragged B) are checked against the
fp64 CPU oracle (oracle/farmer_oracle.py, itself pinned to the same fixtures).
Tolerances (fp32 GPU vs fp32 torch / fp64 oracle): values and loss 1e-5 relative; gradients
|d| <= 1e-5 max|ref| + 1e-4 |ref| per tensor; parameters after the step |d| <= 1e-5 max|p|
(Adam-family steps at positions whose gradient is not ~0, see farmer_golden.well_conditioned).
"""
import numpy as np
import pytest

from farmer_golden import cases, compare_blob, load

pytestmark = pytest.mark.gpu


def _model(B, T, loss="mse", opt="adam", lr=1e-3, params=None):
    from freeimpala_amd.farmer import FarmerLstmModel
    return FarmerLstmModel(batch_size=B, seq_length=T, loss=loss, optimizer=opt, lr=lr, params=params)


@pytest.mark.parametrize("path", cases(), ids=lambda p: p.split("/")[-1][:-4])
def test_farmer_step_vs_reference_golden(path):
    from oracle import farmer_oracle as fo
    g = load(path)
    B, T = int(g["B"]), int(g["T"])
    M = _model(B, T, str(g["loss_kind"]), str(g["optimizer"]), float(g["lr"]), fo.gen_params(int(g["param_seed"])))
    offs = fo.offsets()
    for s in range(int(g["steps"])):
        loss, val = M.train_step(g["z"], g["x"], g["y"], with_values=True)
        np.testing.assert_allclose(val, g[f"step{s}/value"], rtol=1e-5, atol=1e-6)
        ref = float(g[f"step{s}/loss"])
        assert abs(loss - ref) <= 1e-5 * max(1.0, abs(ref)), (loss, ref)
        compare_blob(g, s, "grad", M.get_grads(), offs, rtol=1e-4, atol_frac=1e-5, what="gpu grad")
        compare_blob(g, s, "param", M.get_params(), offs, rtol=1e-6, atol_frac=1e-5, what="gpu param",
                     adam=str(g["optimizer"]) != "sgd")
    M.close()


def _grad_close(a, b, what):
    """||a - b|| <= 1e-5 ||b|| + 1e-7 sqrt(n): relative L2, with an absolute floor for a gradient
    whose terms cancel (MAE's +-1/B signs over an even batch sum to exactly 0 in fp64, to ~1e-9
    in any fp32 order)"""
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    d = np.linalg.norm(a - b)
    assert d <= 1e-5 * np.linalg.norm(b) + 1e-7 * np.sqrt(b.size), f"{what}: |d| {d:.3e}, |ref| {np.linalg.norm(b):.3e}"


@pytest.mark.parametrize("B,T,loss", [(64, 100, "mse"), (13, 1, "huber"), (40, 33, "mae"),
                                      (301, 7, "mse"), (601, 5, "huber"), (1030, 3, "mse")])
def test_farmer_step_vs_oracle_long_and_ragged(B, T, loss):
    """T = 100 (SURVEY.md section 6's CPU measurement shape), T = 1, and the three shapes of the
    register-resident recurrence kernels -- R = 1 row per workgroup (B <= 256), R = 2 (B <= 512:
    301 leaves a half-empty last workgroup), R = 4 (601, 1030: ragged last workgroups, 1030 more
    workgroups than CUs): every gradient tensor within 1e-5 relative L2 of the oracle (absolute
    floor 1e-7 sqrt(n) for cancelling sums)."""
    from oracle import farmer_oracle as fo
    p0 = fo.gen_params(5)
    z, x, y = fo.gen_inputs(6, B, T)
    M = _model(B, T, loss, "sgd", 1e-2, p0)
    lv, val = M.train_step(z, x, y, with_values=True)
    v_ref, saved = fo.forward(p0, z, x)
    l_ref, dval = fo.loss_and_grad(v_ref, y, loss)
    g_ref = fo.backward(p0, saved, dval)
    np.testing.assert_allclose(val, v_ref, rtol=1e-5, atol=1e-6)
    assert abs(lv - l_ref) <= 1e-5 * max(1.0, abs(l_ref))
    g = M.get_grads()
    acts_gpu = [M.tensor_array(f"act{l}", (B, 512)) for l in range(1, 6)]
    for l in range(1, 6):
        e = np.abs(acts_gpu[l - 1] - saved["acts"][l]).max() / max(1.0, np.abs(saved["acts"][l]).max())
        assert e <= 1e-5, (l, e)
    # the fully independent fp64 backward wherever the GPU's ReLU masks (and, for mae, the signs
    # of the residuals) equal fp64's -- then only rounding separates the two gradients
    same_masks = all(np.array_equal(acts_gpu[l - 1] > 0, saved["acts"][l] > 0) for l in range(1, 6))
    same_signs = loss != "mae" or np.array_equal(np.sign(val.astype(np.float64) - y), np.sign(v_ref - y))
    if same_masks and same_signs:
        for n, (a, b, s) in fo.offsets().items():
            _grad_close(g[a:b], g_ref[a:b], n + " (independent fp64 backward)")
    elif B <= 64:
        pytest.fail("a ReLU mask / residual sign differs from fp64 at a small shape: the independent check did not run")
    # the backward fed with the GPU's own dense activations: identical ReLU masks (at B in the
    # hundreds an fp32 pre-activation within ~1e-7 of 0 lands on the other side of the mask than
    # fp64's and moves one row of a weight gradient); the activations themselves are checked above
    saved_gpu = dict(saved, acts=[saved["acts"][0]] + [a.astype(np.float64) for a in acts_gpu])
    g_ref = fo.backward(p0, saved_gpu, dval)
    for n, (a, b, s) in fo.offsets().items():
        _grad_close(g[a:b], g_ref[a:b], n)
    # SGD: p1 = p0 - lr g exactly as torch's p.add_(g, alpha=-lr)
    p1 = M.get_params()
    np.testing.assert_allclose(p1, p0 + np.float32(-1e-2) * g, rtol=0, atol=1e-7)
    M.close()


@pytest.mark.parametrize("B,T", [(301, 9), (601, 6)])
def test_farmer_register_recurrence_is_deterministic(B, T):
    """The R = 2 / R = 4 register-resident recurrences, run on handles created after the device
    memory was filled with NaN garbage: every handle gives bit-identical values and gradients
    (no read of uninitialised memory, no race between the item and matvec phases)."""
    from freeimpala_amd import hip
    from oracle import farmer_oracle as fo
    junk = [hip.DeviceBuffer(64 << 20) for _ in range(4)]
    for j in junk:
        j.upload(np.full((64 << 20) // 4, np.nan, np.float32))
    for j in junk:
        j.free()
    p0 = fo.gen_params(9)
    z, x, y = fo.gen_inputs(10, B, T)
    res = []
    for _ in range(3):
        M = _model(B, T, "mse", "sgd", 1e-2, p0)
        lv, val = M.train_step(z, x, y, with_values=True)
        res.append((lv, val.copy(), M.get_grads()))
        M.close()
    v_ref, _ = fo.forward(p0, z, x)
    np.testing.assert_allclose(res[0][1], v_ref, rtol=1e-5, atol=1e-6)
    for lv, val, g in res[1:]:
        assert lv == res[0][0]
        np.testing.assert_array_equal(val, res[0][1])
        np.testing.assert_array_equal(g, res[0][2])


def test_farmer_forward_equals_train_values_and_is_deterministic():
    from oracle import farmer_oracle as fo
    B, T = 24, 12
    p0 = fo.gen_params(9)
    z, x, y = fo.gen_inputs(10, B, T)
    M1, M2 = _model(B, T, params=p0), _model(B, T, params=p0)
    fwd = M1(z, x, return_value=True)["values"]
    _, val = M1.train_step(z, x, y, with_values=True)
    np.testing.assert_array_equal(fwd, val)
    for _ in range(3):  # M1: 1 + 3 steps, M2: 3 + 1
        M1.train_step(z, x, y)
        M2.train_step(z, x, y)
    M2.train_step(z, x, y)
    np.testing.assert_array_equal(M1.get_params(), M2.get_params())
    M1.close()
    M2.close()


def test_farmer_reference_interface_and_loss_decreases():
    """run_single_training_iteration / get_loss_function / get_optimizer as gpu_benchmark.py,
    on a resident-size default config (B = 32, T = 10); the loss falls over 30 Adam steps on
    a fixed batch."""
    from freeimpala_amd import farmer
    from oracle import farmer_oracle as fo
    z, x, t = farmer.generate_synthetic_data(32, 10, seed=3)
    M = farmer.FarmerLstmModel(32, 10, params=fo.gen_params(3))
    crit, opt = farmer.get_loss_function("mse"), farmer.get_optimizer("adam", None, 1e-3)
    losses = [farmer.run_single_training_iteration(M, z, x, t, crit, opt, None)[1] for _ in range(30)]
    assert losses[-1] < 0.5 * losses[0], losses
    with pytest.raises(ValueError):
        farmer.get_loss_function("hinge")
    with pytest.raises(ValueError):
        farmer.run_single_training_iteration(M, z, x, t, farmer.get_loss_function("mae"), opt, None)
    M.close()


@pytest.mark.parametrize("B,T,loss", [(32, 10, "mse"), (7, 4, "huber"), (64, 5, "mae"), (33, 3, "mse")])
def test_fused_small_batch_torso_matches_layer_kernels(B, T, loss, monkeypatch):
    """B <= 64 runs the torso + head as one grid-synchronised launch per direction
    (mlp_fwd_small / mlp_bwd_small, 128 workgroups, five grid barriers each); FI_FARMER_UNFUSED
    forces the per-layer GEMM path. Same step on both: values and loss 1e-5, every gradient
    tensor within 1e-5 relative L2 (different fp32 summation order), and the fused step
    repeats bit for bit (fixed-order partial sums, no atomics on data)."""
    from oracle import farmer_oracle as fo
    p0 = fo.gen_params(21)
    z, x, y = fo.gen_inputs(22, B, T)
    out = {}
    for mode in ("unfused", "fused", "fused2"):
        if mode == "unfused":
            monkeypatch.setenv("FI_FARMER_UNFUSED", "1")
        else:
            monkeypatch.delenv("FI_FARMER_UNFUSED", raising=False)
        M = _model(B, T, loss, "sgd", 1e-2, p0)
        lv, val = M.train_step(z, x, y, with_values=True)
        out[mode] = (lv, val, M.get_grads(), M.get_params())
        M.close()
    (lu, vu, gu, _), (lf, vf, gf, pf), (l2, v2, g2, p2) = out["unfused"], out["fused"], out["fused2"]
    np.testing.assert_allclose(vf, vu, rtol=1e-5, atol=1e-6)
    assert abs(lf - lu) <= 1e-5 * max(1.0, abs(lu))
    for n, (a, b, s) in fo.offsets().items():
        _grad_close(gf[a:b], gu[a:b], n)
    assert lf == l2
    np.testing.assert_array_equal(vf, v2)
    np.testing.assert_array_equal(gf, g2)
    np.testing.assert_array_equal(pf, p2)


def test_fused_torso_barrier_timeout_is_contained(monkeypatch):
    """a grid barrier of the fused small-batch torso that gives up must not corrupt the
    model. Fault injection (FI_FARMER_SYNC_SKEW) makes the first fused launch's barriers
    unreachable. The two asynchronous steps that follow (no stats: nothing read back) must skip
    their optimizer updates; the next synchronous call reports the timeout once and the parameters
    are still the initial ones. The handle then recovers: its next steps equal a clean twin's,
    bit for bit (same step count for Adam's bias correction)."""
    from freeimpala_amd import farmer
    from freeimpala_amd._abi import FiError
    from oracle import farmer_oracle as fo
    B, T = 32, 4
    z, x, t = farmer.generate_synthetic_data(B, T, seed=11)
    p0 = fo.gen_params(5)
    monkeypatch.setenv("FI_FARMER_SYNC_SKEW", "100000")
    M = _model(B, T, params=p0)
    monkeypatch.delenv("FI_FARMER_SYNC_SKEW")
    twin = _model(B, T, params=p0)
    M.upload_inputs(z, x, t)
    M.train_step_resident(stats=False)
    M.train_step_resident(stats=False)
    with pytest.raises(FiError, match="timed out"):
        M.get_params()
    np.testing.assert_array_equal(M.get_params(), p0.astype(np.float32))
    for _ in range(2):
        l_m, v_m = M.train_step(z, x, t, with_values=True)
        l_t, v_t = twin.train_step(z, x, t, with_values=True)
        assert l_m == l_t
        np.testing.assert_array_equal(v_m, v_t)
        np.testing.assert_array_equal(M.get_params(), twin.get_params())
    M.close()
    twin.close()
