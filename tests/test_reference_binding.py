"""INTEGRATION.md section 2's three-line alias on the reference's OWN classes.

`tests/cpp/reference_binding.cpp` includes `/root/reference/include/freeimpala/
data_structures.h` and `metrics_tracker.h` in place (nothing of the reference is copied) and
instantiates `freeimpala_amd::BasicLearner<SharedBuffer, ModelManager, MetricsTracker>` on the
reference's global-namespace types, exactly as the patched `include/freeimpala/learner.h`
would. Compile flags (Makefile `build/reference_binding`): `-I/root/reference/include
-Itests/cpp/stubs -include optional` (data_structures.h:141 uses std::optional without the
include; `tests/cpp/stubs/spdlog/spdlog.h` stands in for the FetchContent'd spdlog).

CPU (build container): the alias compiles and links against libfi_learner.so, and the
9-argument constructor (learner.h:100-110) reaches the loud "no device" error -- no fallback.
GPU: the binary built here travels to the box (the reference tree does not); the alias learner
and freeimpala_amd::Learner step the same record-schema entries through start() / the worker
loop / stop() and must publish bit-identical blobs; the alias's checkpoint files must hold the
published weights, and --starting-model must resume them.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "build", "reference_binding")
MPI_EXE = os.path.join(ROOT, "build", "reference_mpi_check")
REF = "/root/reference/include/freeimpala/data_structures.h"
MPIEXEC = shutil.which("mpiexec", path="/opt/conda/bin") or shutil.which("mpiexec")


def _mpirun(n, argv, timeout):
    env = dict(os.environ, HYDRA_LAUNCHER="fork")
    return subprocess.run([MPIEXEC, "-n", str(n)] + argv, capture_output=True, text=True, timeout=timeout, env=env)


def _mpi_exe():
    if MPIEXEC is None:
        pytest.skip("no mpiexec (MPICH) in this image")
    if os.path.exists(REF):
        subprocess.run(["make", "-s", "-C", ROOT, "build/reference_mpi_check"], check=True)
    if not os.path.exists(MPI_EXE):
        pytest.skip("build/reference_mpi_check not built (needs the reference headers at build time)")
    return MPI_EXE


def test_alias_compiles_on_reference_classes_and_fails_loudly_without_device():
    if not os.path.exists(REF):
        pytest.skip("reference tree absent (the alias is compiled in the build container only)")
    import torch
    if torch.cuda.is_available():
        pytest.skip("no-device mode expects no GPU")
    subprocess.run(["make", "-s", "-C", ROOT, "build/reference_binding"], check=True)
    r = subprocess.run([EXE, "nodevice"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 3, r.stdout + r.stderr
    assert "no device" in r.stdout and "hipGetDeviceCount" in r.stdout, r.stdout


@pytest.mark.gpu
def test_alias_learner_on_reference_classes_matches_own_classes(tmp_path):
    if not os.path.exists(EXE):
        pytest.skip("build/reference_binding not built (needs the reference headers at build time)")
    r = subprocess.run([EXE, "run", str(tmp_path)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "reference_binding: ok" in r.stdout


# mpi::LearnerEndpoint<SharedBuffer, ModelManager> on the reference's
# own classes (tests/cpp/reference_mpi_check.cpp). (ranks, slots, processors): one receive slot
# and one processor make the path FIFO end to end, which the check then asserts per actor.
@pytest.mark.parametrize("ranks,slots,procs", [(3, 1, 1), (5, 128, 8)])
def test_mpi_endpoint_on_reference_classes_protocol(ranks, slots, procs, tmp_path):
    r = _mpirun(ranks, [_mpi_exe(), "protocol", str(tmp_path), str(slots), str(procs)], timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert f"OK reference_mpi protocol actors={ranks - 1} slots={slots} processors={procs}" in r.stdout


@pytest.mark.parametrize("ranks,slots,procs", [(3, 128, 8), (5, 1, 1)])
def test_mpi_endpoint_feeds_from_reference_agents(ranks, slots, procs, tmp_path):
    """Actor ranks run the reference's own Agent (agent.h with USE_MPI), as
    mpi_async_pool/main.cpp:437-460 does; rank 0 runs the patched receiver."""
    r = _mpirun(ranks, [_mpi_exe(), "agents", str(tmp_path), str(slots), str(procs)], timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert f"OK reference_mpi agents actors={ranks - 1}" in r.stdout


@pytest.mark.gpu
def test_patched_mpi_async_pool_rank0_on_reference_classes(tmp_path):
    """The whole patched rank 0 on the GPU: the section 2 alias Learner on the reference classes
    plus the endpoint, two actor ranks writing record-schema entries."""
    if MPIEXEC is None or not os.path.exists(MPI_EXE):
        pytest.skip("needs mpiexec and build/reference_mpi_check (built in the build container)")
    r = _mpirun(3, [MPI_EXE, "learner", str(tmp_path)], timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK reference_mpi learner actors=2 iterations=3" in r.stdout
