"""GPU parity of the whole MLP learner step (config #2 shape) against the CPU oracle.

forward (fp32 MFMA) -> V-trace/loss -> backward -> optimizer, all through the C ABI
(libfi_learner.so). Tolerance for fp32 tensors: max|d| <= 1e-5 * max(1, max|ref|) per tensor.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def scaled_close(a, b, tol=1e-5, what=""):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    assert np.isfinite(a).all(), what
    s = max(1.0, float(np.abs(b).max()))
    err = float(np.abs(a - b).max()) / s
    assert err <= tol, f"{what}: scaled err {err:.3e}"


def grads_close(a, b, what="", rel_l2=1e-5, rel_max=3e-4):
    """fp32 GEMM gradients vs the fp64 oracle: reductions over (T+1)*B rows accumulate in fp32
    (MFMA), so elementwise error scales with sum|terms|, not |result|. Criterion per tensor:
    ||d||_2 <= rel_l2 ||ref||_2 and max|d| <= rel_max * max|ref|."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    assert np.isfinite(a).all(), what
    l2 = np.linalg.norm(a - b) / max(1e-30, np.linalg.norm(b))
    mx = np.abs(a - b).max() / max(1e-30, np.abs(b).max())
    assert l2 <= rel_l2 and mx <= rel_max, f"{what}: rel L2 {l2:.2e}, rel max {mx:.2e}"


def mk(T=5, B=16, A=18, D=128, H=256, arch="mlp", **kw):
    from freeimpala_amd.learner import DeviceLearner
    kw.setdefault("optimizer", "sgd")
    kw.setdefault("lr", 1e-3)
    kw.setdefault("max_grad_norm", 0.0)
    if arch != "mlp":
        return DeviceLearner(arch, seq_len=T, batch=B, num_actions=A, **kw)
    return DeviceLearner("mlp", seq_len=T, batch=B, num_actions=A, obs_dim=D, hidden=H, **kw)


def oracle_step(orc, L, batch, p0, gpu_acts=False):
    """Oracle forward -> V-trace -> backward. gpu_acts=True feeds the oracle backward with the
    GPU's own h1/h2 and upstream gradient (identical ReLU masks), isolating the backward."""
    T, B, A, D, H = L.T, L.B, L.A, L.D, L.H
    obs = batch["obs"].reshape((T + 1) * B, D)
    h1, h2, out = orc.mlp_forward(obs, p0, H=H, A=A)
    if gpu_acts:
        h1, h2 = L.tensor("h1", shape=h1.shape), L.tensor("h2", shape=h2.shape)
    logits = out[:, :A].reshape(T + 1, B, A)
    values = out[:, A].reshape(T + 1, B)
    vt = orc.vtrace_loss(logits[:T], batch["mu"], batch["actions"], batch["rewards"],
                         batch["discounts"], values)
    dout = np.zeros(((T + 1) * B, A + 1), np.float32)
    if gpu_acts:
        dout[:T * B, :A] = L.tensor("dlogits").reshape(T * B, A)
        dout[:, A] = L.tensor("dvalue")
    else:
        dout[:T * B, :A] = vt["dlogits"].reshape(T * B, A)
        dout[:, A] = vt["dvalue"].reshape(-1)
    g = orc.mlp_backward(obs, p0, h1, h2, dout, H=H, A=A)
    return dict(logits=logits, values=values, vt=vt, grads=g, h1=h1, h2=h2)


def test_synth_bit_exact_vs_oracle(orc):
    L = mk(T=6, B=16, D=32, H=32)
    L.synth(seed=1234, b_global=64, b_offset=16)
    ref = orc.synth_batch(1234, T=6, B=16, A=18, D=32, B_glob=64, b_off=16)
    np.testing.assert_array_equal(L.tensor("obs", shape=(7, 16, 32)), ref["obs"])
    np.testing.assert_array_equal(L.tensor("mu", shape=(6, 16, 18)), ref["mu"])
    np.testing.assert_array_equal(L.tensor("actions", np.int32, (6, 16)), ref["actions"])
    np.testing.assert_array_equal(L.tensor("rewards", shape=(6, 16)), ref["rewards"])
    np.testing.assert_array_equal(L.tensor("discounts", shape=(6, 16)), ref["discounts"])


@pytest.mark.parametrize("T,B", [(5, 16), (20, 48)])
def test_mlp_step_parity(orc, T, B):
    L = mk(T=T, B=B)
    L.synth(seed=7)
    batch = orc.synth_batch(7, T=T, B=B, A=18, D=128)
    p0 = L.get_params()
    st = L.step_resident()
    ref = oracle_step(orc, L, batch, p0)
    scaled_close(L.tensor("logits", shape=(T + 1, B, 18)), ref["logits"], what="logits")
    scaled_close(L.tensor("values", shape=(T + 1, B)), ref["values"], what="values")
    scaled_close(L.tensor("vs", shape=(T, B)), ref["vt"]["vs"], what="vs")
    scaled_close(L.tensor("dlogits", shape=(T, B, 18)), ref["vt"]["dlogits"], what="dlogits")
    g = L.tensor("grads")
    D, H, A = 128, 256, 18
    off = np.cumsum([0, D * H, H, H * H, H, H * (A + 1), A + 1])
    for i, name in enumerate(["W1", "b1", "W2", "b2", "Wh", "bh"]):
        grads_close(g[off[i]:off[i + 1]], ref["grads"][off[i]:off[i + 1]], what=name)
    tot = ref["vt"]["losses"]
    assert abs(st["pg_loss"] - tot[0]) <= 1e-5 * max(1, abs(tot[0]))
    assert abs(st["baseline_loss"] - tot[1]) <= 1e-5 * max(1, abs(tot[1]))
    assert abs(st["entropy_loss"] - tot[2]) <= 1e-5 * max(1, abs(tot[2]))
    np.testing.assert_allclose(st["grad_norm"], np.linalg.norm(ref["grads"].astype(np.float64)),
                               rtol=1e-5)
    # SGD, no clipping: p1 = p0 - lr * g
    scaled_close(L.get_params(), p0 - np.float32(1e-3) * g, 1e-6, "sgd update")
    assert st["version"] == 1


@pytest.mark.parametrize("D,H,A,T,B", [(17, 48, 4, 3, 24), (1, 5, 2, 2, 16), (128, 1000, 33, 2, 40),
                                       (64, 512, 64, 3, 16), (100, 130, 7, 4, 8)])
def test_mlp_other_shapes_parity(orc, D, H, A, T, B):
    """MLP shapes away from config #2 (every obs_dim / hidden / action count the create call
    accepts is a legal configuration): odd widths that cut the fp32 MFMA tiles (hidden 5, 48,
    130, 1000), a one-float observation, A up to the 64-action limit, B not a multiple of 16.
    Forward, V-trace, every gradient and the SGD update against the oracle."""
    L = mk(T=T, B=B, A=A, D=D, H=H)
    L.synth(seed=D * 7 + H)
    batch = orc.synth_batch(D * 7 + H, T=T, B=B, A=A, D=D)
    p0 = L.get_params()
    st = L.step_resident()
    ref = oracle_step(orc, L, batch, p0)
    scaled_close(L.tensor("logits", shape=(T + 1, B, A)), ref["logits"], what="logits")
    scaled_close(L.tensor("values", shape=(T + 1, B)), ref["values"], what="values")
    scaled_close(L.tensor("dlogits", shape=(T, B, A)), ref["vt"]["dlogits"], what="dlogits")
    g = L.tensor("grads")
    off = np.cumsum([0, D * H, H, H * H, H, H * (A + 1), A + 1])
    assert g.size == off[-1]
    for i, name in enumerate(["W1", "b1", "W2", "b2", "Wh", "bh"]):
        grads_close(g[off[i]:off[i + 1]], ref["grads"][off[i]:off[i + 1]], what=name)
    tot = orc.total_loss(ref["vt"]["losses"])
    assert abs(st["total_loss"] - tot) <= 1e-5 * max(1.0, abs(tot))
    scaled_close(L.get_params(), p0 - np.float32(1e-3) * g, 1e-6, "sgd update")
    L.close()


def test_mlp_config2_full_size(orc):
    """Config #2: T=100, B=512, A=18, obs 128, MLP 128-256-256, fp32 numerics vs the oracle."""
    T, B = 100, 512
    L = mk(T=T, B=B)
    L.synth(seed=42)
    batch = orc.synth_batch(42, T=T, B=B, A=18, D=128)
    p0 = L.get_params()
    L.step_resident()
    ref = oracle_step(orc, L, batch, p0, gpu_acts=True)
    h1, h2, _ = orc.mlp_forward(batch["obs"].reshape(-1, 128), p0)
    scaled_close(L.tensor("h1", shape=h1.shape), h1, what="h1")
    scaled_close(L.tensor("h2", shape=h2.shape), h2, what="h2")
    scaled_close(L.tensor("vs", shape=(T, B)), ref["vt"]["vs"], what="vs")
    scaled_close(L.tensor("pg_adv", shape=(T, B)), ref["vt"]["pg_adv"], what="pg_adv")
    scaled_close(L.tensor("dlogits", shape=(T, B, 18)), ref["vt"]["dlogits"], what="dlogits")
    scaled_close(L.tensor("dvalue", shape=(T + 1, B)), ref["vt"]["dvalue"], what="dvalue")
    g = L.tensor("grads")
    D, H, A = 128, 256, 18
    off = np.cumsum([0, D * H, H, H * H, H, H * (A + 1), A + 1])
    for i, name in enumerate(["W1", "b1", "W2", "b2", "Wh", "bh"]):
        grads_close(g[off[i]:off[i + 1]], ref["grads"][off[i]:off[i + 1]], what=name)


def test_adam_and_clip_match_oracle(orc):
    L = mk(T=4, B=16, optimizer="adam", lr=5e-4, max_grad_norm=1.0)
    L.synth(seed=3)
    p0 = L.get_params()
    st = L.step_resident()
    g = L.tensor("grads")
    p = p0.copy()
    gg = g.copy()
    norm = orc.clip_grad_norm(gg, 1.0)
    np.testing.assert_allclose(st["grad_norm"], norm, rtol=1e-6)
    m = np.zeros_like(p)
    v = np.zeros_like(p)
    orc.adam(p, gg, m, v, 5e-4, 0.9, 0.999, 1e-8, 1)
    scaled_close(L.get_params(), p, 1e-6, "adam params")
    scaled_close(L.tensor("adam_m"), m, 1e-6, "adam m")


def test_host_entries_step_equals_resident_step(orc):
    """SharedBuffer entries (host bytes, record schema) -> ingest kernel -> same step."""
    from freeimpala_amd.learner import pack_records
    T, B = 8, 32
    batch = orc.synth_batch(11, T=T, B=B, A=18, D=128)
    entries = pack_records(batch["obs"], batch["mu"], batch["actions"], batch["rewards"],
                           batch["discounts"], entry_size=T + 3)
    L1, L2 = mk(T=T, B=B, seed=5), mk(T=T, B=B, seed=5)
    L1.synth(seed=11)
    s1 = L1.step_resident()
    s2 = L2.step(entries)
    np.testing.assert_array_equal(L2.tensor("obs"), L1.tensor("obs"))
    np.testing.assert_array_equal(L2.tensor("actions", np.int32), L1.tensor("actions", np.int32))
    np.testing.assert_array_equal(L2.get_params(), L1.get_params())
    assert s1["total_loss"] == s2["total_loss"]


def test_publish_blob_and_resume():
    L = mk(T=3, B=16, publish="bf16")
    assert L.param_bytes == 2 * L.param_count
    L.synth(seed=1)
    L.step_resident()
    blob, ver = L.get_blob()
    assert ver == 1 and len(blob) == L.param_bytes
    L2 = mk(T=3, B=16, seed=99)
    L2.set_params(blob, version=ver)
    p1 = L.get_params()
    p2 = L2.get_params()
    # bf16 round trip: |d| <= 2^-8 relative
    assert np.all(np.abs(p2 - p1) <= np.abs(p1) * 2 ** -8 + 1e-30)


def test_loss_decreases_over_steps():
    """gamma = 0: the V-trace target is the clipped immediate reward, so the value loss of a
    fixed batch is a regression that SGD must reduce."""
    L = mk(T=10, B=64, optimizer="sgd", lr=1e-4, max_grad_norm=40.0, gamma=0.0)
    L.synth(seed=5)
    base = [L.step_resident()["baseline_loss"] for _ in range(30)]
    assert base[-1] < 0.9 * base[0]


def test_bad_arguments_fail_loudly():
    from freeimpala_amd._abi import FiError
    L = mk(T=3, B=16)
    with pytest.raises(FiError):
        L.step([b"\0" * 1024] * 16)  # entries shorter than (T+1)*1024
    with pytest.raises(FiError):
        L.step([b"\0" * 4096] * 15)  # wrong batch size


def oracle_sgd_trajectory(orc, L, raw_batches, p0, lr=1e-3):
    """The oracle's view of len(raw_batches) SGD steps from p0: final parameters and the last
    step's total loss (computed with the parameters before that step)."""
    p = p0.astype(np.float32).copy()
    tot = None
    for b in raw_batches:
        ref = oracle_step(orc, L, b, p)
        tot = orc.total_loss(ref["vt"]["losses"])
        p = (p - np.float32(lr) * ref["grads"].astype(np.float32)).astype(np.float32)
    return p, tot


@pytest.mark.parametrize("opt", ["adam", "sgd"])
def test_async_step_matches_sync_steps(orc, opt):
    """fi_learner_step_async x4 (entries freed right after each call; both staging slots are
    reused, so the H2D of batch k+2 must wait for the ingest of batch k) then wait == four
    synchronous steps on the same batches: same parameters, same last statistics. With SGD the
    run is also replayed through the oracle (forward, V-trace, backward, update per batch):
    final parameters and the last step's loss match it."""
    from freeimpala_amd.learner import pack_records
    T, B = 6, 32
    batches, raw = [], []
    for seed in (21, 22, 23, 24):
        b = orc.synth_batch(seed, T=T, B=B, A=18, D=128)
        raw.append(b)
        batches.append(pack_records(b["obs"], b["mu"], b["actions"], b["rewards"], b["discounts"],
                                    entry_size=T + 1))
    L1, L2 = mk(T=T, B=B, seed=9, optimizer=opt), mk(T=T, B=B, seed=9, optimizer=opt)
    p0 = L2.get_params()
    for e in batches:
        s1 = L1.step(e)
    for e in batches:
        ent = [bytes(x) for x in e]
        L2.step_async(ent)
        del ent  # the call copied them
    s2 = L2.wait()
    np.testing.assert_array_equal(L1.get_params(), L2.get_params())
    assert s1["total_loss"] == s2["total_loss"] and s1["version"] == s2["version"] == 4
    if opt == "sgd":
        p_ref, tot = oracle_sgd_trajectory(orc, L2, raw, p0)
        scaled_close(L2.get_params(), p_ref, 1e-6, "params after 4 async steps vs oracle")
        assert abs(s2["total_loss"] - tot) <= 1e-5 * max(1.0, abs(tot)), (s2["total_loss"], tot)


@pytest.mark.parametrize("opt", ["adam", "sgd"])
def test_staged_steps_match_entry_steps(orc, opt):
    """Zero-copy staging: batches written straight into the acquired pinned buffer (what
    SharedBuffer::readBatchInto would do), submitted sync and async, give the same parameters
    and statistics as fi_learner_step on the same entries. Submitting without an acquired
    buffer is an error that leaves the handle usable. With SGD the five steps are also replayed
    through the oracle: final parameters and the last loss match it."""
    from freeimpala_amd._abi import FiError
    from freeimpala_amd.learner import pack_records
    T, B = 6, 32
    batches, raw = [], []
    for seed in (31, 32, 33, 34, 35):
        b = orc.synth_batch(seed, T=T, B=B, A=18, D=128)
        raw.append(b)
        batches.append(pack_records(b["obs"], b["mu"], b["actions"], b["rewards"], b["discounts"],
                                    entry_size=T + 2))  # one spare record: S > T+1
    L1, L2 = mk(T=T, B=B, seed=4, optimizer=opt), mk(T=T, B=B, seed=4, optimizer=opt)
    p0 = L2.get_params()
    for e in batches:
        s1 = L1.step(e)
    with pytest.raises(FiError):
        L2.step_staged()
    for i, e in enumerate(batches):
        dst = L2.acquire_staging()
        assert dst.shape == (B, (T + 1) * 1024)
        assert L2.acquire_staging().ctypes.data == dst.ctypes.data  # same buffer until submitted
        for j, x in enumerate(e):
            dst[j] = np.frombuffer(x, np.uint8)[:dst.shape[1]]
        if i == 0:
            L2.step_staged(stats=False)
        else:
            L2.step_staged_async()
    s2 = L2.wait()
    np.testing.assert_array_equal(L1.get_params(), L2.get_params())
    assert s1["total_loss"] == s2["total_loss"] and s1["version"] == s2["version"] == 5
    if opt == "sgd":
        p_ref, tot = oracle_sgd_trajectory(orc, L2, raw, p0)
        scaled_close(L2.get_params(), p_ref, 1e-6, "params after 5 staged steps vs oracle")
        assert abs(s2["total_loss"] - tot) <= 1e-5 * max(1.0, abs(tot)), (s2["total_loss"], tot)


@pytest.mark.parametrize("arch", ["mlp", "atari"])
@pytest.mark.parametrize("attach", ["uid", "init_all"])
def test_rccl_one_rank_allreduce_step_matches(monkeypatch, arch, attach):
    """The data-parallel path on one GPU: a handle attached to a one-rank RCCL communicator
    (FI_COMM_SINGLE) runs the bucketed in-step ncclAllReduce(sum) of the gradient (3 buckets,
    reverse layer order, on the comm stream overlapped with the backward); a one-rank sum is
    the identity, so its parameters after three Adam steps equal those of a handle without a
    communicator, bit for bit. Covers unique id / attach (one-rank-per-process form and the
    grouped single-process fi_comm_init_all) / all-reduce / teardown, and RCCL's own view of
    the communicator; N > 1 needs several GPUs (RCCL refuses two ranks on one device)."""
    from freeimpala_amd.learner import DeviceLearner
    monkeypatch.setenv("FI_COMM_SINGLE", "1")
    kw = dict(T=4, B=32, seed=5, optimizer="adam")
    if arch == "atari":
        kw = dict(T=2, B=16, seed=5, optimizer="adam")
    L1, L2 = mk(arch=arch, **kw), mk(arch=arch, **kw)
    if attach == "uid":
        L2.attach_comm(DeviceLearner.comm_unique_id(), 0, 1)
    else:
        DeviceLearner.comm_init_all([L2])
    assert L1.comm_info()["nranks"] == 1
    s = {}
    for i, L in enumerate((L1, L2)):
        L.synth(seed=12)
        for _ in range(3):
            s[i] = L.step_resident()
    np.testing.assert_array_equal(L1.get_params(), L2.get_params())
    assert s[0]["total_loss"] == s[1]["total_loss"]
    assert L2.comm_info() == {"nranks": 1, "rank": 0, "buckets_last_step": 3}
    assert L1.comm_info()["buckets_last_step"] == 0
    L1.close()
    L2.close()


def test_state_checkpoint_resume_is_bit_exact():
    """save_state after one step, load it into a fresh learner, step both on the same batch:
    identical parameters and Adam moments (optimizer state restored, not just weights)."""
    L1 = mk(T=5, B=16, optimizer="adam", seed=3)
    L1.synth(seed=8)
    L1.step_resident()
    blob = L1.save_state()
    L2 = mk(T=5, B=16, optimizer="adam", seed=77)
    L2.synth(seed=8)
    L2.load_state(blob)
    np.testing.assert_array_equal(L1.get_params(), L2.get_params())
    a, b = L1.step_resident(), L2.step_resident()
    np.testing.assert_array_equal(L1.get_params(), L2.get_params())
    np.testing.assert_array_equal(L1.tensor("adam_v"), L2.tensor("adam_v"))
    assert a["version"] == b["version"] == 2
    from freeimpala_amd._abi import FiError
    with pytest.raises(FiError):
        L2.load_state(blob[:-4])


def test_out_of_range_action_rejects_batch(orc):
    """A record whose action lies outside [0, A) (corrupt entry, or actors run with another
    --num-actions) is not clamped into a plausible gradient: the step returns FI_ERR_INVALID,
    the parameters, Adam moments and version stay as they were, and the next valid batch
    steps normally (the oracle rejects the same batch with -3). Sync, async and staged forms."""
    from freeimpala_amd._abi import FiError
    from freeimpala_amd.learner import pack_records
    T, B = 4, 32
    good = orc.synth_batch(41, T=T, B=B, A=18, D=128)
    bad = {k: (None if v is None else v.copy()) for k, v in good.items()}
    bad["actions"][2, 5] = 18
    bad["actions"][0, 0] = -1
    with pytest.raises(Exception):
        orc.vtrace_loss(np.zeros((T, B, 18), np.float32), bad["mu"], bad["actions"], bad["rewards"],
                        bad["discounts"], np.zeros((T + 1, B), np.float32))
    pk = lambda b: pack_records(b["obs"], b["mu"], b["actions"], b["rewards"], b["discounts"],
                                entry_size=T + 1)
    L, R = mk(T=T, B=B, seed=6, optimizer="adam"), mk(T=T, B=B, seed=6, optimizer="adam")
    R.step(pk(good))
    L.step(pk(good))
    p1, m1 = L.get_params(), L.tensor("adam_m")
    with pytest.raises(FiError, match="outside"):
        L.step(pk(bad))
    np.testing.assert_array_equal(L.get_params(), p1)
    np.testing.assert_array_equal(L.tensor("adam_m"), m1)
    L.step_async(pk(bad))
    with pytest.raises(FiError, match="outside"):
        L.wait()
    np.testing.assert_array_equal(L.get_params(), p1)
    s = L.step(pk(good))
    r = R.step(pk(good))
    assert s["version"] == r["version"] == 2
    np.testing.assert_array_equal(L.get_params(), R.get_params())


@pytest.mark.parametrize("attach", ["uid", "init_all"])
def test_rejected_batch_under_comm_leaves_state_unchanged(orc, monkeypatch, attach):
    """With a communicator attached the reject decision is all-reduced (a one-int
    ncclAllReduce(sum) of the bad-action counter after the last gradient bucket) and the
    optimizer reads the reduced flag, so every replica skips a batch that any shard rejects.
    On one GPU (FI_COMM_SINGLE one-rank communicator, both attach forms): a bad batch through
    the in-step all-reduce path raises FI_ERR_INVALID and leaves parameters, both Adam moments
    and the version bit-unchanged; the next good batch then matches a handle without a
    communicator bit for bit."""
    from freeimpala_amd._abi import FiError
    from freeimpala_amd.learner import DeviceLearner, pack_records
    monkeypatch.setenv("FI_COMM_SINGLE", "1")
    T, B = 4, 32
    good = orc.synth_batch(43, T=T, B=B, A=18, D=128)
    bad = {k: (None if v is None else v.copy()) for k, v in good.items()}
    bad["actions"][3, 31] = 18
    pk = lambda b: pack_records(b["obs"], b["mu"], b["actions"], b["rewards"], b["discounts"],
                                entry_size=T + 1)
    L, R = mk(T=T, B=B, seed=6, optimizer="adam"), mk(T=T, B=B, seed=6, optimizer="adam")
    if attach == "uid":
        L.attach_comm(DeviceLearner.comm_unique_id(), 0, 1)
    else:
        DeviceLearner.comm_init_all([L])
    L.step(pk(good))
    R.step(pk(good))
    p1, m1, v1 = L.get_params(), L.tensor("adam_m"), L.tensor("adam_v")
    with pytest.raises(FiError, match="outside"):
        L.step(pk(bad))
    np.testing.assert_array_equal(L.get_params(), p1)
    np.testing.assert_array_equal(L.tensor("adam_m"), m1)
    np.testing.assert_array_equal(L.tensor("adam_v"), v1)
    assert L.comm_info()["buckets_last_step"] == 3
    s, r = L.step(pk(good)), R.step(pk(good))
    assert s["version"] == r["version"] == 2
    np.testing.assert_array_equal(L.get_params(), R.get_params())
    L.close()
    R.close()


@pytest.mark.parametrize("attach", [None, "uid"])
@pytest.mark.parametrize("poison", [np.nan, np.inf])
def test_nonfinite_gradient_skips_update(orc, monkeypatch, attach, poison):
    """A NaN / Inf reward (a corrupt record) makes the losses and the summed gradient
    non-finite. The gradient-norm kernel flags it (the norm is taken from the all-reduced
    gradient, so every replica sees the same flag) and the optimizer skips the update: the
    step returns FI_ERR_NONFINITE (-7), parameters, both Adam moments and the version stay
    bit-unchanged, and the next good batch matches a handle that never saw the bad one. Sync
    and async forms; with and without the in-step all-reduce path (one-rank communicator)."""
    from freeimpala_amd._abi import FiError
    from freeimpala_amd.learner import DeviceLearner, pack_records
    monkeypatch.setenv("FI_COMM_SINGLE", "1")
    T, B = 4, 32
    good = orc.synth_batch(47, T=T, B=B, A=18, D=128)
    bad = {k: (None if v is None else v.copy()) for k, v in good.items()}
    bad["rewards"][1, 7] = poison
    pk = lambda b: pack_records(b["obs"], b["mu"], b["actions"], b["rewards"], b["discounts"],
                                entry_size=T + 1)
    L, R = mk(T=T, B=B, seed=6, optimizer="adam"), mk(T=T, B=B, seed=6, optimizer="adam")
    if attach:
        L.attach_comm(DeviceLearner.comm_unique_id(), 0, 1)
    L.step(pk(good))
    R.step(pk(good))
    p1, m1, v1 = L.get_params(), L.tensor("adam_m"), L.tensor("adam_v")
    with pytest.raises(FiError, match=r"rc=-7.*not finite"):
        L.step(pk(bad))
    L.step_async(pk(bad))
    with pytest.raises(FiError, match="not finite"):
        L.wait()
    np.testing.assert_array_equal(L.get_params(), p1)
    np.testing.assert_array_equal(L.tensor("adam_m"), m1)
    np.testing.assert_array_equal(L.tensor("adam_v"), v1)
    s, r = L.step(pk(good)), R.step(pk(good))
    assert s["version"] == r["version"] == 2
    assert np.isfinite(s["grad_norm"]) and s["total_loss"] == r["total_loss"]
    np.testing.assert_array_equal(L.get_params(), R.get_params())
    L.close()
    R.close()


@pytest.mark.parametrize("kind", ["action", "nan"])
def test_skipped_step_behind_others_in_flight_is_reported(orc, kind):
    """Three asynchronous steps enqueued back to back (no wait between them), the middle batch
    bad (an out-of-range action, or a NaN reward). The device counts the skipped update, so the
    wait after the third step reports it (the flags of the last step alone are clean), the
    version counts the two applied updates (also when published before the wait: it never goes
    back), and the parameters equal a handle that stepped
    only the two good batches (SGD: no step-number dependence), bit for bit."""
    from freeimpala_amd._abi import FiError
    from freeimpala_amd.learner import pack_records
    T, B = 4, 32
    good1 = orc.synth_batch(61, T=T, B=B, A=18, D=128)
    good2 = orc.synth_batch(62, T=T, B=B, A=18, D=128)
    bad = {k: (None if v is None else v.copy()) for k, v in good1.items()}
    if kind == "action":
        bad["actions"][2, 9] = 18
    else:
        bad["rewards"][0, 3] = np.nan
    pk = lambda b: pack_records(b["obs"], b["mu"], b["actions"], b["rewards"], b["discounts"],
                                entry_size=T + 1)
    L, R = mk(T=T, B=B, seed=8), mk(T=T, B=B, seed=8)
    v0 = L.step(pk(good1))["version"]
    R.step(pk(good1))
    for b in (good2, bad, good1):
        L.step_async(pk(b))
    # publication before the wait sees the completed steps and counts applied updates only
    assert L.get_blob()[1] == v0 + 2
    with pytest.raises(FiError, match="outside" if kind == "action" else "not finite"):
        L.wait()
    assert L.get_blob()[1] == v0 + 2
    R.step(pk(good2))
    r = R.step(pk(good1))
    np.testing.assert_array_equal(L.get_params(), R.get_params())
    s = L.step(pk(good2))  # the handle carries on; the skip counter was cleared by the wait
    assert s["version"] == r["version"] + 1 == v0 + 3
    L.close()
    R.close()


def _two_devices():
    from freeimpala_amd import hip
    n = hip.device_count()
    if n < 2:
        pytest.skip(f"needs 2 GPUs (this box has {n}): RCCL refuses two ranks on one device")


def test_two_device_data_parallel_matches_full_batch_and_oracle(orc):
    """Batch-dim data parallelism on two devices (single process, fi_comm_init_all, one thread
    per device as DeviceLearner::step_sharded runs it): each replica steps its half of the
    batch, the in-step all-reduce sums the two shard gradients, so both replicas end with
    identical parameters equal to one device stepping the whole batch, and to the oracle's
    SGD step on the full batch (sum order across the shards differs: 1e-6 scaled). Skipped on
    one-GPU boxes; kept ready for the first multi-GPU run."""
    from concurrent.futures import ThreadPoolExecutor
    from freeimpala_amd.learner import DeviceLearner, pack_records
    _two_devices()
    T, B = 4, 32
    b = orc.synth_batch(51, T=T, B=B, A=18, D=128)
    pk = lambda sl: pack_records(b["obs"][:, sl], b["mu"][:, sl], b["actions"][:, sl], b["rewards"][:, sl],
                                 b["discounts"][:, sl], entry_size=T + 1)
    halves = [slice(0, B // 2), slice(B // 2, B)]
    full = mk(T=T, B=B, seed=6)
    reps = [mk(T=T, B=B // 2, seed=6, device=d) for d in (0, 1)]
    DeviceLearner.comm_init_all(reps)
    assert [r.comm_info()["nranks"] for r in reps] == [2, 2]
    p0 = full.get_params()
    for r in reps:
        np.testing.assert_array_equal(r.get_params(), p0)
    st = full.step(pk(slice(None)))
    with ThreadPoolExecutor(2) as ex:
        res = list(ex.map(lambda i: reps[i].step(pk(halves[i])), (0, 1)))
    np.testing.assert_array_equal(reps[0].get_params(), reps[1].get_params())
    scaled_close(reps[0].get_params(), full.get_params(), 1e-6, "2-device vs 1-device params")
    ref = oracle_step(orc, full, b, p0)
    scaled_close(reps[0].get_params(), p0 - np.float32(1e-3) * ref["grads"], 1e-6, "2-device vs oracle SGD")
    assert abs((res[0]["total_loss"] + res[1]["total_loss"]) - st["total_loss"]) <= 1e-5 * max(1, abs(st["total_loss"]))
    for r in reps + [full]:
        r.close()


def test_two_device_atari_bucketed_overlap_matches_full_batch():
    """The Atari network on two devices: the three gradient buckets (fc + heads, conv3,
    conv1 + conv2) are all-reduced on the comm stream while the conv backward still runs, so
    the overlapped path gets a real peer. Each replica synthesises its half of the global batch
    (columns indexed globally), both end bit-identical, and equal to one device stepping the
    whole batch up to the order of the fp32 gradient sums (per-frame activations are
    grid-independent, the slab reductions are not). Skipped on one-GPU boxes."""
    from concurrent.futures import ThreadPoolExecutor
    from freeimpala_amd.learner import DeviceLearner
    _two_devices()
    T, B = 2, 32
    full = mk(arch="atari", T=T, B=B, seed=6)
    reps = [mk(arch="atari", T=T, B=B // 2, seed=6, device=d) for d in (0, 1)]
    DeviceLearner.comm_init_all(reps)
    full.synth(seed=12, b_global=B, b_offset=0)
    for i, r in enumerate(reps):
        r.synth(seed=12, b_global=B, b_offset=i * B // 2)
    p0 = full.get_params()
    for r in reps:
        np.testing.assert_array_equal(r.get_params(), p0)
    for _ in range(2):
        st = full.step_resident()
        with ThreadPoolExecutor(2) as ex:
            res = list(ex.map(lambda i: reps[i].step_resident(), (0, 1)))
        assert abs(res[0]["total_loss"] + res[1]["total_loss"] - st["total_loss"]) <= 1e-5 * max(1, abs(st["total_loss"]))
    assert [r.comm_info()["buckets_last_step"] for r in reps] == [3, 3]
    np.testing.assert_array_equal(reps[0].get_params(), reps[1].get_params())
    scaled_close(reps[0].get_params(), full.get_params(), 1e-6, "2-device vs 1-device Atari params")
    for r in reps + [full]:
        r.close()


@pytest.mark.parametrize("nproc", [1, 2])
@pytest.mark.parametrize("arch", ["mlp", "atari"])
def test_two_process_attach_comm_matches_single_device(arch, nproc, tmp_path):
    """bench.py's N > 1 form: processes under torch.distributed.run, one device each, the
    RCCL unique id broadcast over gloo, fi_learner_attach_comm, SGD steps with the in-step
    all-reduce (tests/dist_attach_worker.py). Replicas bit-identical; equal to one device
    stepping the whole batch (1e-6 scaled); the shard losses sum to the full batch's.
    nproc=2 is skipped on one-GPU boxes; nproc=1 runs the same script on one GPU with a
    one-rank communicator (FI_COMM_SINGLE), so the launcher path is exercised everywhere."""
    import json
    import os
    import socket
    import subprocess
    import sys
    if nproc == 2:
        _two_devices()
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(root, "tests", "dist_attach_worker.py"), "--arch", arch, "--out", str(tmp_path)]
    env = dict(os.environ, FI_COMM_SINGLE="1") if nproc == 1 else None
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=root, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = json.loads((tmp_path / "result.json").read_text())
    assert res["world"] == nproc and res["comm"]["nranks"] == nproc and res["buckets_last_step"] == 3
    assert res["replicas_identical"]
    assert res["max_scaled_diff_vs_one_device"] <= 1e-6, res
    for a, b in zip(res["loss_sum"], res["one_device_loss"]):
        assert abs(a - b) <= 1e-5 * max(1.0, abs(b)), res


def test_two_device_reject_is_agreed(orc):
    """A bad action in ONE replica's shard: the all-reduced reject flag makes BOTH replicas
    skip the optimizer (both raise FI_ERR_INVALID, parameters and version unchanged on both), so
    they stay identical. Skipped on one-GPU boxes."""
    from concurrent.futures import ThreadPoolExecutor
    from freeimpala_amd._abi import FiError
    from freeimpala_amd.learner import DeviceLearner, pack_records
    _two_devices()
    T, B = 4, 16
    good = orc.synth_batch(52, T=T, B=2 * B, A=18, D=128)
    bad = {k: (None if v is None else v.copy()) for k, v in good.items()}
    bad["actions"][1, B + 3] = 18  # in replica 1's half only
    pk = lambda d, sl: pack_records(d["obs"][:, sl], d["mu"][:, sl], d["actions"][:, sl], d["rewards"][:, sl],
                                    d["discounts"][:, sl], entry_size=T + 1)
    halves = [slice(0, B), slice(B, 2 * B)]
    reps = [mk(T=T, B=B, seed=9, optimizer="adam", device=d) for d in (0, 1)]
    DeviceLearner.comm_init_all(reps)

    def run(d, i):
        try:
            return reps[i].step(pk(d, halves[i]))
        except FiError as e:
            return e
    with ThreadPoolExecutor(2) as ex:
        list(ex.map(lambda i: run(good, i), (0, 1)))
    p1 = [r.get_params() for r in reps]
    with ThreadPoolExecutor(2) as ex:
        out = list(ex.map(lambda i: run(bad, i), (0, 1)))
    assert all(isinstance(o, FiError) for o in out), out
    for r, p in zip(reps, p1):
        np.testing.assert_array_equal(r.get_params(), p)
    np.testing.assert_array_equal(reps[0].get_params(), reps[1].get_params())
    for r in reps:
        r.close()
