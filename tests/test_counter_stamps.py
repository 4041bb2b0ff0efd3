"""The roofline counter fields belong to the timed build: bench.py attaches a
committed PMC summary only when its `_build.source_hash` equals the hash of the sources it runs
from, and the hash covers exactly the learner step's sources. CPU only (no device involved)."""
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_source_hash_covers_the_learner_sources_only():
    from freeimpala_amd import build_info
    files = [os.path.relpath(f, ROOT) for f in build_info.source_files()]
    assert "include/fi_learner.h" in files and "Makefile" in files
    assert "freeimpala_amd/csrc/vtrace.hip" in files and "freeimpala_amd/csrc/atari_fr.hip" in files
    # the FarmerLstm step never runs inside the learner step: its kernels do not change the hash
    assert "freeimpala_amd/csrc/farmer.hip" not in files
    h = build_info.source_hash()
    assert len(h) == 16 and h == build_info.source_hash()
    assert build_info.stamp({"arch": "x"}) == {"source_hash": h, "runtime": build_info.runtime_key(), "arch": "x"}


def _fake_root(tmp_path, stamp):
    """a copy of the tree's profiles/ with only our fake counter files, bench.ROOT pointed at it"""
    (tmp_path / "profiles").mkdir()
    for kind, body in (("traffic", {"conv21_bwd": {"hbm_bytes_per_launch": 123}}),
                       ("mfma", {"conv21_bwd": {"mfma_util": 0.5}})):
        from freeimpala_amd import build_info
        d = dict(body, _build={"source_hash": stamp, "runtime": build_info.runtime_key()})
        (tmp_path / "profiles" / f"zz_pmc_{kind}_atari.json").write_text(json.dumps(d))
    return str(tmp_path)


def test_bench_attaches_counters_of_this_build(tmp_path, monkeypatch):
    import bench
    from freeimpala_amd import build_info
    monkeypatch.setattr(bench, "ROOT", _fake_root(tmp_path, build_info.source_hash()))
    tr, mf, info = bench.load_counters("atari", (100, 4096, 18))
    assert tr == {"conv21_bwd": 123} and mf["conv21_bwd"]["mfma_util"] == 0.5
    assert info["traffic_file"].endswith("zz_pmc_traffic_atari.json")


def test_bench_refuses_counters_of_another_build(tmp_path, monkeypatch):
    import bench
    monkeypatch.setattr(bench, "ROOT", _fake_root(tmp_path, "0123456789abcdef"))
    tr, mf, info = bench.load_counters("atari", (100, 4096, 18))
    assert tr == {} and mf == {} and info["traffic_file"] is None and "no counter pass" in info["note"]


def test_bench_refuses_counters_of_another_shape(tmp_path, monkeypatch):
    import bench
    from freeimpala_amd import build_info
    monkeypatch.setattr(bench, "ROOT", _fake_root(tmp_path, build_info.source_hash()))
    tr, mf, info = bench.load_counters("atari", (100, 512, 18))
    assert tr == {} and mf == {} and "T=100 B=4096" in info["note"]


def test_bench_refuses_counters_taken_under_other_switches(tmp_path, monkeypatch):
    """the same sources run different kernels under FI_* switches (e.g.
    FI_BWD_UNFUSED): a pass stamped under one setting is not attached to a line timed under
    another."""
    import bench
    from freeimpala_amd import build_info
    monkeypatch.delenv("FI_BWD_UNFUSED", raising=False)
    monkeypatch.setattr(bench, "ROOT", _fake_root(tmp_path, build_info.source_hash()))
    monkeypatch.setenv("FI_BWD_UNFUSED", "1")
    tr, mf, info = bench.load_counters("atari", (100, 4096, 18))
    assert tr == {} and mf == {} and info["runtime"]["env"] == {"FI_BWD_UNFUSED": "1"}
