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
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "build", "reference_binding")
REF = "/root/reference/include/freeimpala/data_structures.h"


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
