"""The drop-in Learner surface (include/freeimpala_amd/learner.hpp) and the cmd/freeimpala-
shaped binary on it (tools/fi_freeimpala.cpp).

CPU: replay buffer / model store / flag semantics (tests/cpp/replay_check.cpp); the binary
parses the reference's command line strictly, with the learner flags registered; without a
GPU it fails loudly (no CPU fallback).
GPU: BASELINE config #1 (--players 1 --iterations 32 --buffer-capacity 32 --batch-size 32
--seq-length 100 --agents 4, entries of T+1 = 101 records) end to end: 4 producer threads ->
SharedBuffer -> readBatchInto pinned staging -> device step -> ModelManager publication ->
checkpoints every c; the learner iteration count is floor(A * iterations / M) = 4
(reference cmd/freeimpala/main.cpp:179); every consumed batch is replayed through the CPU
oracle and every published parameter version checked against it; then a second run resumes
from the checkpoint directory (--starting-model) with the optimizer state.
"""
import json
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "build", "fi_freeimpala")
CHK = os.path.join(ROOT, "build", "replay_check")

CONFIG1 = ["--players", "1", "--iterations", "32", "--buffer-capacity", "32", "--batch-size", "32",
           "--seq-length", "100", "--agents", "4", "--entry-size", "101", "--game-steps", "101"]


def _make(target, exe):
    srcs = [os.path.join(ROOT, "tools", "fi_freeimpala.cpp"), os.path.join(ROOT, "tests", "cpp", "replay_check.cpp")]
    srcs += [os.path.join(ROOT, "include", "freeimpala_amd", f)
             for f in os.listdir(os.path.join(ROOT, "include", "freeimpala_amd"))]
    # rebuild a stale binary only where the tree can build (here: build/obj exists); the GPU
    # box runs the binaries built beforehand and shipped with the tree
    stale = os.path.exists(exe) and os.path.isdir(os.path.join(ROOT, "build", "obj")) and \
        os.path.getmtime(exe) < max(os.path.getmtime(s) for s in srcs)
    if not os.path.exists(exe) or stale:
        subprocess.run(["make", "-s", "-C", ROOT, target], check=True)
    return exe


def run(args, timeout=300):
    return subprocess.run([_make("tools", EXE)] + args, capture_output=True, text=True, timeout=timeout)


def test_replay_buffer_model_store_and_flags(tmp_path):
    r = subprocess.run([_make("host", CHK), str(tmp_path / "ck")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK replay" in r.stdout


def test_cli_parses_reference_command_line_strictly():
    r = run(["--help"])
    assert r.returncode == 0
    for flag in ("--players", "--iterations", "--buffer-capacity", "--batch-size", "--entry-size",
                 "--agents", "--game-steps", "--learner-time", "--checkpoint-freq", "--seq-length",
                 "--learner-arch", "--lr", "--devices", "--optimizer", "--publish", "--data-parallel"):
        assert flag in r.stdout, flag
    assert run(["--no-such-flag", "3"]).returncode == 1
    assert run(["--players", "two"]).returncode == 1
    assert run(["--log-level", "chatty"]).returncode == 1
    # main.cpp:164-176 validation
    assert run(CONFIG1[:6] + ["--batch-size", "64"]).returncode == 1
    assert run(["--entry-size", "10", "--game-steps", "20"]).returncode == 1
    # --data-parallel G splits each player's M entries over G devices: G must divide M
    assert run(CONFIG1 + ["--data-parallel", "3"]).returncode == 1


def test_cli_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("expects no GPU")
    r = run(CONFIG1 + ["--agent-time", "0"])
    assert r.returncode == 2, r.stdout + r.stderr
    assert "fi_learner_create" in r.stderr and "device" in r.stderr


def _unpack(batch, T, B, A, D):
    rec = batch.reshape(B, T + 1, 1024)
    f = rec.view(np.float32)
    obs = np.ascontiguousarray(f[:, :, :D].transpose(1, 0, 2))
    mu = np.ascontiguousarray(f[:, :T, 128:128 + A].transpose(1, 0, 2))
    act = np.ascontiguousarray(rec[:, :T, 768:772].copy().view(np.int32)[..., 0].T)
    rew = np.ascontiguousarray(f[:, :T, 193].T)
    disc = np.ascontiguousarray(f[:, :T, 194].T)
    return obs, mu, act, rew, disc


def _oracle_sgd_grad(orc, p, batch, T, B, A, D, H):
    obs, mu, act, rew, disc = _unpack(batch, T, B, A, D)
    h1, h2, out = orc.mlp_forward(obs.reshape(-1, D), p, H=H, A=A)
    vt = orc.vtrace_loss(out[:, :A].reshape(T + 1, B, A)[:T], mu, act, rew, disc, out[:, A].reshape(T + 1, B))
    dout = np.zeros(((T + 1) * B, A + 1), np.float32)
    dout[:T * B, :A] = vt["dlogits"].reshape(T * B, A)
    dout[:, A] = vt["dvalue"].reshape(-1)
    return orc.mlp_backward(obs.reshape(-1, D), p, h1, h2, dout, H=H, A=A), vt["losses"]


@pytest.mark.gpu
def test_config1_end_to_end_vs_oracle_and_resume(orc, tmp_path):
    T, B, A, D, H, lr = 100, 32, 18, 128, 256, 1e-3
    ck, dump = tmp_path / "ck", tmp_path / "dump"
    common = ["--agent-time", "0", "--checkpoint-freq", "2", "--checkpoint-location", str(ck),
              "--optimizer", "sgd", "--lr", str(lr), "--max-grad-norm", "0", "--seed", "7"]
    r = run(CONFIG1 + common + ["--dump-dir", str(dump)])
    assert r.returncode == 0, r.stdout + r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["learner_iterations"] == [4] and out["expected_iterations"] == 4
    m = out["metrics"]
    assert m["data_transfers"] == 4 * 32
    assert m["learner_model_updates"] == 4 and m["rejected_batches"] == 0
    assert m["learner_env_steps"] == 4 * T * B
    nbytes = out["param_bytes"]
    # checkpoints: reference file format + optimizer-state sidecars
    for it in (2, 4):
        f = ck / f"model_0_{it}.bin"
        assert f.stat().st_size == 8 + nbytes
        assert (ck / f"model_0_{it}.state").exists()
    latest = np.fromfile(ck / "model_0_latest.bin", np.uint8)
    assert int(latest[:8].view(np.uint64)[0]) == 4
    # replay every consumed batch through the oracle from the published parameters
    p = np.fromfile(dump / "params_0_0.bin", np.float32)
    for k in range(4):
        batch = np.fromfile(dump / f"batch_0_{k}.bin", np.uint8)
        assert batch.size == B * (T + 1) * 1024
        g, _ = _oracle_sgd_grad(orc, p, batch, T, B, A, D, H)
        p1 = np.fromfile(dump / f"params_0_{k + 1}.bin", np.float32)
        g_dev = (p.astype(np.float64) - p1) / lr
        l2 = np.linalg.norm(g_dev - g) / np.linalg.norm(g)
        assert l2 < 2e-3, (k, l2)
        p = p1
    np.testing.assert_array_equal(latest[8:].view(np.float32), p)
    # resume: --starting-model picks model_0_latest.bin + its .state; publication continues at 5.
    # --iterations 64 with 4 agents and M = 32 -> floor(4 * 64 / 32) = 8 learner iterations; the
    # count restarts at 0 after a resume, as in the reference (learner.h:73)
    dump2 = tmp_path / "dump2"
    r = run(CONFIG1[:2] + ["--iterations", "64"] + CONFIG1[4:] + common[:4] + ["--checkpoint-location", str(tmp_path / "ck2")]
            + common[6:] + ["--starting-model", str(ck), "--dump-dir", str(dump2)])
    assert r.returncode == 0, r.stdout + r.stderr
    assert "resumed learner state" in r.stderr
    out2 = json.loads(r.stdout.strip().splitlines()[-1])
    assert out2["learner_iterations"] == [8]
    np.testing.assert_array_equal(np.fromfile(dump2 / "params_0_4.bin", np.float32), p)
    assert (dump2 / "params_0_5.bin").exists() and (dump2 / "params_0_12.bin").exists()
