"""Host code under sanitizers (the reference has none, and latent races).

tests/cpp/race_check.cpp stresses the host side around the learner step from many threads:
SharedBuffer writers / try_writers against readBatch / readBatchInto readers and draining,
ModelManager publication against model copies, version polls, waits and concurrent checkpoint
saves, MetricsTracker counters, and the SimLearner worker / checkpoint threads with actor
threads (config #1's machinery). It is built twice and must finish clean both times:
  * ThreadSanitizer (clang++ from /opt/rocm/lib/llvm: gcc 11's TSAN does not intercept
    pthread_cond_clockwait, which libstdc++'s wait_for uses, and reports false double locks);
  * AddressSanitizer + UndefinedBehaviorSanitizer (g++), every finding fatal.
The TSAN build found a real race on its first run: ModelManager::saveModel read models_[p]
(and the checkpoint counter) unlocked while updateModel wrote it -- the reference's own latent
race (data_structures.h:395,402) carried into the restatement; saveModel now reads through the
locked getModel and the counter is atomic. CPU only, no GPU and no libfi_learner.so.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLANG = "/opt/rocm/lib/llvm/bin/clang++"


# (program, the line it prints when every check holds): the stress above, and the semantic
# checks of the buffer / model store / flag parser (tests/cpp/replay_check.cpp)
PROGRAMS = [("race_check", "OK race"), ("replay_check", "OK replay")]


def _build_and_run(tmp_path, compiler, flags, env_extra, prog="race_check"):
    exe = str(tmp_path / prog)
    src = os.path.join(ROOT, "tests", "cpp", prog + ".cpp")
    cmd = [compiler, "-std=c++17", "-O1", "-g", *flags, "-I" + os.path.join(ROOT, "include"), src,
           "-o", exe, "-pthread"]
    b = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert b.returncode == 0, b.stderr[-4000:]
    env = dict(os.environ, **env_extra)
    r = subprocess.run([exe, str(tmp_path / "work")], capture_output=True, text=True, timeout=600, env=env)
    return r


@pytest.mark.skipif(not os.path.exists(CLANG), reason="no clang++ with the TSAN runtime")
@pytest.mark.parametrize("prog,ok", PROGRAMS)
def test_host_side_is_race_free_under_tsan(tmp_path, prog, ok):
    r = _build_and_run(tmp_path, CLANG, ["-fsanitize=thread"], {"TSAN_OPTIONS": "halt_on_error=1 exitcode=66"}, prog)
    assert "WARNING: ThreadSanitizer" not in r.stderr, r.stderr[-6000:]
    assert r.returncode == 0 and ok in r.stdout, (r.returncode, r.stderr[-3000:])


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
@pytest.mark.parametrize("prog,ok", PROGRAMS)
def test_host_side_clean_under_asan_ubsan(tmp_path, prog, ok):
    r = _build_and_run(tmp_path, "g++", ["-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                                         "-fno-omit-frame-pointer"],
                       {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0", "UBSAN_OPTIONS": "print_stacktrace=1"}, prog)
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-6000:]
    assert r.returncode == 0 and ok in r.stdout, (r.returncode, r.stderr[-3000:])


MPIEXEC = shutil.which("mpiexec", path="/opt/conda/bin")


@pytest.mark.skipif(not os.path.exists(CLANG) or MPIEXEC is None, reason="needs ROCm's clang++ and MPICH")
def test_mpi_endpoint_is_race_free_under_tsan(tmp_path):
    """The rank-0 MPI endpoint (include/freeimpala_amd/mpi_pool.hpp: receiver thread, processor
    pool, per-player buffers, version / weights replies) against 4 actor ranks, every rank built
    with ThreadSanitizer (tests/cpp/mpi_pool_check.cpp, the protocol test of tests/test_mpi.py)."""
    exe = str(tmp_path / "mpi_pool_tsan")
    b = subprocess.run([CLANG, "-std=c++17", "-O1", "-g", "-fsanitize=thread", "-I" + os.path.join(ROOT, "include"),
                        "-I/opt/conda/include", os.path.join(ROOT, "tests", "cpp", "mpi_pool_check.cpp"), "-o", exe,
                        "-pthread", "/opt/conda/lib/libmpi.so", "-Wl,--disable-new-dtags",
                        "-Wl,-rpath,/usr/lib/x86_64-linux-gnu:/opt/conda/lib"], capture_output=True, text=True, timeout=600)
    assert b.returncode == 0, b.stderr[-4000:]
    env = dict(os.environ, HYDRA_LAUNCHER="fork", TSAN_OPTIONS="halt_on_error=1 exitcode=66")
    r = subprocess.run([MPIEXEC, "-n", "5", exe, str(tmp_path / "work")], capture_output=True, text=True,
                       timeout=300, env=env)
    assert "WARNING: ThreadSanitizer" not in r.stdout + r.stderr, (r.stdout + r.stderr)[-6000:]
    assert r.returncode == 0 and "OK mpi_pool actors=4" in r.stdout, (r.stdout + r.stderr)[-3000:]


@pytest.mark.skipif(not os.path.exists(CLANG), reason="no clang++ with the TSAN runtime")
def test_cli_with_sim_learner_is_race_free_under_tsan(tmp_path):
    """build/fi_freeimpala's whole threaded run (tools/fi_freeimpala.cpp: argument parsing, the
    SimLearner's worker and checkpoint threads, 4 actor threads writing entries and syncing the
    model, cleanup and the metrics line) built with ThreadSanitizer; `--learner sim` touches no
    device, so libfi_learner.so is linked but never called."""
    lib = os.path.join(ROOT, "freeimpala_amd", "lib")
    if not os.path.exists(os.path.join(lib, "libfi_learner.so")):
        pytest.skip("libfi_learner.so not built")
    exe = str(tmp_path / "fi_freeimpala_tsan")
    b = subprocess.run([CLANG, "-std=c++17", "-O1", "-g", "-fsanitize=thread", "-I" + os.path.join(ROOT, "include"),
                        os.path.join(ROOT, "tools", "fi_freeimpala.cpp"), "-o", exe, "-pthread", "-L" + lib,
                        "-lfi_learner", "-Wl,-rpath," + lib, "-Wl,-rpath,/opt/rocm/lib"],
                       capture_output=True, text=True, timeout=600)
    assert b.returncode == 0, b.stderr[-4000:]
    r = subprocess.run([exe, "--learner", "sim", "--players", "2", "--iterations", "16", "--buffer-capacity", "8",
                        "--batch-size", "4", "--agents", "4", "--learner-time", "0", "--agent-time", "0",
                        "--entry-size", "8", "--game-steps", "8", "--seq-length", "3", "--checkpoint-freq", "2",
                        "--checkpoint-location", str(tmp_path / "ck")],
                       capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66"))
    assert "WARNING: ThreadSanitizer" not in r.stderr, r.stderr[-6000:]
    assert r.returncode == 0, r.stderr[-3000:]
    assert '"learner_iterations": [16, 16]' in r.stdout


TSAN_BIN = os.path.join(ROOT, "build", "tsan")
SUPP = os.path.join(ROOT, "tests", "tsan_rocm.supp")


def _tsan_env():
    return dict(os.environ, TSAN_OPTIONS=f"halt_on_error=0 exitcode=66 suppressions={SUPP}")


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(os.path.join(TSAN_BIN, "host_learner_check")),
                    reason="build/tsan not built (make -f tests/cpp/tsan.mk)")
def test_device_host_paths_race_free_under_tsan(tmp_path):
    """The host side of the DEVICE learner under ThreadSanitizer on the GPU, the library's own
    host code (csrc/learner.cpp) instrumented too (build/tsan/lib, tests/cpp/tsan.mk); the ROCm
    runtime, uninstrumented, is suppressed (its own thread synchronisation is invisible to TSAN):
      * tests/cpp/host_learner_check.cpp gpu -- two players stepping concurrently through the
        C ABI from their own threads (DeviceLearner, pinned staging, async H2D);
      * host_learner_check pipeline -- 139 MB batches copied by the library's staging threads,
        three asynchronous steps back to back beside a synchronous twin on another thread;
      * build/fi_freeimpala with the device learner -- 2 players, 4 actor threads, the
        BasicLearner worker and checkpoint threads, model sync, stop()."""
    r = subprocess.run([os.path.join(TSAN_BIN, "host_learner_check"), "gpu", str(tmp_path / "hlc")],
                       capture_output=True, text=True, timeout=300, env=_tsan_env())
    assert "WARNING: ThreadSanitizer" not in r.stderr, r.stderr[-6000:]
    assert r.returncode == 0 and "OK gpu" in r.stdout, (r.returncode, r.stdout[-2000:], r.stderr[-3000:])
    r = subprocess.run([os.path.join(TSAN_BIN, "host_learner_check"), "pipeline"],
                       capture_output=True, text=True, timeout=300, env=_tsan_env())
    assert "WARNING: ThreadSanitizer" not in r.stderr, r.stderr[-6000:]
    assert r.returncode == 0 and "OK pipeline" in r.stdout, (r.returncode, r.stdout[-2000:], r.stderr[-3000:])
    r = subprocess.run([os.path.join(TSAN_BIN, "fi_freeimpala"), "--players", "2", "--iterations", "32",
                        "--buffer-capacity", "32", "--batch-size", "16", "--seq-length", "20", "--agents", "4",
                        "--entry-size", "42", "--game-steps", "42", "--agent-time", "0", "--checkpoint-freq", "2",
                        "--checkpoint-location", str(tmp_path / "ck")],
                       capture_output=True, text=True, timeout=300, env=_tsan_env())
    assert "WARNING: ThreadSanitizer" not in r.stderr, r.stderr[-6000:]
    assert r.returncode == 0 and '"learner_iterations": [8, 8]' in r.stdout, (r.returncode, r.stderr[-3000:])


ASAN_BIN = os.path.join(ROOT, "build", "asan")


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(os.path.join(ASAN_BIN, "host_learner_check")),
                    reason="build/asan not built (make -f tests/cpp/tsan.mk)")
def test_device_host_paths_clean_under_asan_ubsan(tmp_path):
    """The same device host paths under AddressSanitizer + UBSan, the library's host side
    (csrc/learner.cpp) instrumented as well (build/asan/lib): two players stepping concurrently,
    the pipelined 139 MB batches through the staging threads, and the threaded CLI on the device
    learner. Every finding is fatal; leak checking is off (the ROCm runtime holds its
    allocations to process exit), and the link-order check is off (the harness preloads a
    library of its own ahead of the sanitizer runtime)."""
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:verify_asan_link_order=0:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    (tmp_path / "hlc").mkdir()
    runs = [[os.path.join(ASAN_BIN, "host_learner_check"), "gpu", str(tmp_path / "hlc")],
            [os.path.join(ASAN_BIN, "host_learner_check"), "pipeline"],
            [os.path.join(ASAN_BIN, "fi_freeimpala"), "--players", "2", "--iterations", "32",
             "--buffer-capacity", "32", "--batch-size", "16", "--seq-length", "20", "--agents", "4",
             "--entry-size", "42", "--game-steps", "42", "--agent-time", "0", "--checkpoint-freq", "2",
             "--checkpoint-location", str(tmp_path / "ck")]]
    for cmd in runs:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
        assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-6000:]
        assert r.returncode == 0, (cmd[1:2], r.returncode, r.stdout[-2000:], r.stderr[-3000:])
