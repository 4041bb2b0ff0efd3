"""bench.py's cpu_baseline choice: one whole B = 4096 Atari CPU step by
default when the host has the memory for it, the bounded extrapolated sample otherwise, and the
line says which and why. CPU only: the decision and the headroom probe, not the 50 s step."""
import bench


def test_full_step_is_the_default_with_headroom():
    assert bench.full_cpu_step("atari", 4096, False, False, 300.0) == (True, None)


def test_sample_when_memory_is_short_and_the_reason_is_reported():
    full, why = bench.full_cpu_step("atari", 4096, False, False, 62.3)
    assert not full and "62.3 GB" in why and str(bench.CPU_FULL_GB) in why
    full, why = bench.full_cpu_step("atari", 4096, False, False, None)
    assert not full and "None" in why


def test_flags_and_shapes():
    assert bench.full_cpu_step("atari", 4096, True, False, 10.0) == (True, None)  # --cpu-full forces it
    assert bench.full_cpu_step("atari", 4096, False, True, 300.0) == (False, "--cpu-sample")
    full, why = bench.full_cpu_step("atari", 512, False, False, 300.0)
    assert not full and "B=512" in why
    assert bench.full_cpu_step("mlp", 4096, False, False, 10.0) == (False, None)  # MLP steps run whole anyway


def test_headroom_probe_reports_a_positive_size():
    room = bench.host_mem_headroom_gb()
    assert room is None or room > 0
