"""C++ host side (include/freeimpala_amd/device_learner.hpp) over the C ABI.

CPU: the check program builds against the header + libfi_learner.so, parses the reference's
learner flags, and fails loudly (no CPU fallback) when no GPU is present.
GPU: two players step the same SharedBuffer-shaped batch from two std::threads; the
program checks both results are identical, and this test checks the step against the CPU
oracle (losses 1e-5 relative, SGD update per tensor as in test_gpu_learner.py).
"""
import json
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "build", "host_learner_check")


def _build():
    src = os.path.join(ROOT, "tests", "cpp", "host_learner_check.cpp")
    if not os.path.exists(EXE) or (os.path.isdir(os.path.join(ROOT, "build", "obj")) and
                                   os.path.getmtime(EXE) < os.path.getmtime(src)):
        subprocess.run(["make", "-s", "-C", ROOT, "host"], check=True)
    return EXE


def test_host_cpp_cpu_mode():
    import torch
    if torch.cuda.is_available():
        pytest.skip("cpu mode expects no GPU")
    r = subprocess.run([_build(), "cpu"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK cpu" in r.stdout


def _unpack(batch, T, B, S, A, D):
    rec = batch.reshape(B, S, 1024)[:, :T + 1]
    f = rec.view(np.float32)  # (B, T+1, 256)
    obs = np.ascontiguousarray(f[:, :, :D].transpose(1, 0, 2))
    mu = np.ascontiguousarray(f[:, :T, 128:128 + A].transpose(1, 0, 2))
    act = np.ascontiguousarray(rec[:, :T, 768:772].copy().view(np.int32)[..., 0].T)
    rew = np.ascontiguousarray(f[:, :T, 193].T)
    disc = np.ascontiguousarray(f[:, :T, 194].T)
    return obs, mu, act, rew, disc


@pytest.mark.gpu
def test_host_cpp_two_players_vs_oracle(orc, tmp_path):
    r = subprocess.run([_build(), "gpu", str(tmp_path)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    st = json.loads((tmp_path / "stats.json").read_text())
    T, B, S, A, D = st["T"], st["B"], st["S"], st["A"], st["D"]
    batch = np.fromfile(tmp_path / "batch.bin", np.uint8)
    p0 = np.fromfile(tmp_path / "params0.bin", np.float32)
    p1 = np.fromfile(tmp_path / "params1.bin", np.float32)
    obs, mu, act, rew, disc = _unpack(batch, T, B, S, A, D)
    H = 256
    _, _, out = orc.mlp_forward(obs.reshape(-1, D), p0, H=H, A=A)
    logits = out[:, :A].reshape(T + 1, B, A)
    values = out[:, A].reshape(T + 1, B)
    vt = orc.vtrace_loss(logits[:T], mu, act, rew, disc, values)
    for i, k in enumerate(["pg_loss", "baseline_loss", "entropy_loss"]):
        ref = vt["losses"][i]
        assert abs(st[k] - ref) <= 1e-5 * max(1.0, abs(ref)), (k, st[k], ref)
    # SGD, no clipping: p1 = p0 - lr * g  -> recovered gradient vs the oracle's
    h1, h2, _ = orc.mlp_forward(obs.reshape(-1, D), p0, H=H, A=A)
    dout = np.zeros(((T + 1) * B, A + 1), np.float32)
    dout[:T * B, :A] = vt["dlogits"].reshape(T * B, A)
    dout[:, A] = vt["dvalue"].reshape(-1)
    g = orc.mlp_backward(obs.reshape(-1, D), p0, h1, h2, dout, H=H, A=A)
    g_dev = (p0.astype(np.float64) - p1) / st["lr"]
    l2 = np.linalg.norm(g_dev - g) / np.linalg.norm(g)
    assert l2 < 2e-3, l2  # recovered through an fp32 parameter difference
    np.testing.assert_allclose(st["grad_norm"], np.linalg.norm(g.astype(np.float64)), rtol=1e-4)


@pytest.mark.gpu
def test_worker_failure_drains_buffer_and_releases_actors(tmp_path):
    """a worker whose staging acquisition fails stops, reports workerFailed(), and
    drains its buffer, so an actor blocked in SharedBuffer::write returns (false) instead of
    hanging the run."""
    r = subprocess.run([_build(), "worker_fail", str(tmp_path)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK worker_fail" in r.stdout
