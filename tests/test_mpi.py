"""MPI feeding of the learner (include/freeimpala_amd/mpi_pool.hpp) and the
freeimpala_mpi_async_pool-shaped binary on it (tools/fi_freeimpala_mpi.cpp), BASELINE config #5.

CPU: the wire protocol under mpiexec with a stand-in learner (tests/cpp/mpi_pool_check.cpp):
every trajectory arrives once and intact in its player's buffer, version / weights replies
carry `u64 version || blob` of the published model (reference agent.h:76-151,
mpi_async_pool/main.cpp:243-357); the binary parses the reference command line and, without
a GPU, rank 0 fails loudly and takes the actor ranks down (no CPU fallback).
GPU: 4 actor ranks feeding the device learner on rank 0 with config #1's sizes (M=32, T=100,
S=101): the learner iteration count floor(A * iterations / M), the endpoint's counts, and every
consumed batch replayed through the CPU oracle against the published parameter versions.
"""
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

from test_dropin import CONFIG1, _make, assert_step_matches_oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MPIEXEC = shutil.which("mpiexec", path="/opt/conda/bin") or shutil.which("mpiexec")
EXE = os.path.join(ROOT, "build", "fi_freeimpala_mpi")
CHK = os.path.join(ROOT, "build", "mpi_pool_check")

pytestmark = pytest.mark.skipif(MPIEXEC is None, reason="no mpiexec (MPICH) in this image")


def mpirun(n, argv, timeout=300):
    env = dict(os.environ, HYDRA_LAUNCHER="fork")
    return subprocess.run([MPIEXEC, "-n", str(n)] + argv, capture_output=True, text=True, timeout=timeout, env=env)


@pytest.mark.parametrize("ranks", [2, 5])
def test_mpi_pool_protocol(ranks, tmp_path):
    r = mpirun(ranks, [_make("build/mpi_pool_check", CHK), str(tmp_path)], timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert f"OK mpi_pool actors={ranks - 1}" in r.stdout


def test_mpi_cli_parses_and_fails_loudly_without_gpu():
    exe = _make("build/fi_freeimpala_mpi", EXE)
    r = mpirun(1, [exe, "--help"], timeout=60)
    assert r.returncode == 0
    for flag in ("--players", "--iterations", "--batch-size", "--entry-size", "--seq-length", "--learner-arch"):
        assert flag in r.stdout, flag
    assert mpirun(2, [exe, "--no-such-flag", "1"], timeout=60).returncode == 1
    import torch
    if torch.cuda.is_available():
        return
    r = mpirun(3, [exe] + CONFIG1 + ["--agent-time", "0"], timeout=120)
    assert r.returncode != 0
    assert "fi_learner_create" in r.stderr


@pytest.mark.gpu
def test_config5_shape_mpi_end_to_end_vs_oracle(orc, tmp_path):
    """4 actor ranks -> rank-0 receiver -> SharedBuffer -> device learner -> weights over tags
    200/210; every consumed batch replayed through the oracle (SGD: the published parameter
    difference / lr is the gradient)."""
    T, B, A, D, H, lr = 100, 32, 18, 128, 256, 1e-3
    ck, dump = tmp_path / "ck", tmp_path / "dump"
    args = CONFIG1 + ["--agent-time", "0", "--checkpoint-freq", "2", "--checkpoint-location", str(ck),
                      "--optimizer", "sgd", "--lr", str(lr), "--max-grad-norm", "0", "--seed", "11",
                      "--dump-dir", str(dump)]
    r = mpirun(5, [EXE] + args, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["expected_iterations"] == 4 and out["learner_iterations"] == [4]
    m = out["mpi"]
    assert m["actors"] == 4 and m["trajectories"] == 4 * 32
    assert m["trajectory_bytes"] == 4 * 32 * 101 * 1024
    assert m["version_requests"] == 4 * 32 and m["bad_messages"] == 0
    assert m["weights_replies"] >= 1
    assert m["weights_bytes"] == m["weights_replies"] * (8 + out["param_bytes"])
    assert out["metrics"]["learner_model_updates"] == 4 and out["metrics"]["rejected_batches"] == 0
    p = np.fromfile(dump / "params_0_0.bin", np.float32)
    for k in range(4):
        p = assert_step_matches_oracle(orc, dump, k, p, T, B, A, D, H, lr)
    latest = np.fromfile(ck / "model_0_latest.bin", np.uint8)
    assert int(latest[:8].view(np.uint64)[0]) == 4
    np.testing.assert_array_equal(latest[8:].view(np.float32), p)


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_config5_64_actor_ranks_end_to_end(orc, tmp_path):
    """BASELINE config #5's rank count: 64 MPI actor ranks on the host cores feeding the device
    learner on rank 0 (one GPU here; the 8-GPU form needs an 8-GPU node). 64 x 16 trajectories
    of T = 100 (105 MB) through the rank-0 receiver into the SharedBuffer; the learner runs
    floor(64 * 16 / 256) = 4 iterations at M = 256. Every message arrives once and intact, every
    actor's version request is answered, weight replies carry whole blobs, and the first consumed batch is replayed through the
    oracle (SGD: its published parameter difference / lr is the gradient)."""
    T, B, A, D, H, lr, actors, iters = 100, 256, 18, 128, 256, 1e-3, 64, 16
    dump = tmp_path / "dump"
    args = ["--players", "1", "--iterations", str(iters), "--buffer-capacity", str(2 * B), "--batch-size", str(B),
            "--seq-length", str(T), "--entry-size", str(T + 1), "--game-steps", str(T + 1), "--agent-time", "0",
            "--checkpoint-freq", "0", "--checkpoint-location", str(tmp_path / "ck"), "--optimizer", "sgd",
            "--lr", str(lr), "--max-grad-norm", "0", "--seed", "5", "--dump-dir", str(dump), "--log-level", "warn"]
    r = mpirun(actors + 1, [EXE] + args, timeout=280)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["expected_iterations"] == actors * iters // B and out["learner_iterations"] == [actors * iters // B]
    m = out["mpi"]
    assert m["actors"] == actors and m["trajectories"] == actors * iters and m["bad_messages"] == 0
    assert m["trajectory_bytes"] == actors * iters * (T + 1) * 1024
    assert m["version_requests"] == actors * iters
    assert m["weights_bytes"] == m["weights_replies"] * (8 + out["param_bytes"])
    assert out["metrics"]["rejected_batches"] == 0
    p = np.fromfile(dump / "params_0_0.bin", np.float32)
    assert_step_matches_oracle(orc, dump, 0, p, T, B, A, D, H, lr)
