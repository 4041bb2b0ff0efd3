"""bench.py's step_roofline: the step's HBM bytes are the stamped PMC
bytes of every kernel of the step, summed; every kernel's gap to its floor is listed by gap."""
import json
import os

import pytest

from freeimpala_amd.atari_shapes import atari_kernel_work
from freeimpala_amd.roofline import step_roofline

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PMC = os.path.join(ROOT, "profiles", "r05u_pmc_traffic_atari.json")
MFMA = os.path.join(ROOT, "profiles", "r05u_pmc_mfma_atari.json")
BENCH = os.path.join(ROOT, "profiles", "r05t_bench_atari.json")


def _load(p):
    with open(p) as fh:
        return {k: v for k, v in json.load(fh).items() if not k.startswith("_")}


@pytest.fixture(scope="module")
def inputs():
    tr = {k: v["hbm_bytes_per_launch"] for k, v in _load(PMC).items()}
    mf = _load(MFMA)
    with open(BENCH) as fh:
        b = json.load(fh)
    work = atari_kernel_work(100, 4096, 18)
    work["vtrace"] = (0, (12 * 18 + 28) * 100 * 4096)
    return tr, mf, b["kernel_ms_per_step"], b["ms_per_step"], work


def test_pmc_bytes_sum_over_the_step(inputs):
    tr, mf, kms, ms, work = inputs
    sr = step_roofline(kms, {k: 1 for k in kms}, work, tr, mf, ms)
    in_step = [k for k in kms if k in work]
    expect = sum(tr[k] for k in in_step if k in tr) + sum(work[k][1] for k in in_step if k not in tr)
    assert sr["hbm_bytes_per_step"]["pmc"] == int(expect)
    # the r05 tree: ~86.7 GB counted + heads_fwd (no PMC entry) at its ~0.45 GB algorithmic bytes
    assert sr["hbm_bytes_per_step"]["kernels_at_algorithmic_bytes"] == ["heads_fwd"]
    assert 86.0e9 < sr["hbm_bytes_per_step"]["pmc"] < 88.0e9
    tbs = expect / (ms * 1e-3) / 1e12
    assert sr["achieved_tbs"] == pytest.approx(tbs, abs=1e-3)
    assert sr["frac_of_peak_8tbs"] == pytest.approx(tbs / 8.0, abs=1e-4)
    assert sr["hbm_floor_ms"]["pmc_bytes_at_6p3tbs"] == pytest.approx(expect / 6.3e9, abs=1e-3)
    assert 13.5 < sr["hbm_floor_ms"]["pmc_bytes_at_6p3tbs"] < 14.2   # DESIGN.md's corrected floor
    # every frac below 1, and the floors below the step
    assert sr["frac_of_peak_8tbs"] < 1 and sr["sum_of_kernel_floors_ms"] < ms


def test_kernels_sorted_by_gap_and_floors(inputs):
    tr, mf, kms, ms, work = inputs
    sr = step_roofline(kms, {k: 1 for k in kms}, work, tr, mf, ms)
    rows = sr["kernels_by_gap"]
    gaps = [r["gap_ms"] for r in rows]
    assert gaps == sorted(gaps, reverse=True)
    assert {r["kernel"] for r in rows} == set(kms)
    assert set(sr["unmodelled_kernels"]) == {"reduce_slabs", "weights_bf16", "optimizer", "grad_norm",
                                              "allreduce_wait"}
    row = {r["kernel"]: r for r in rows}
    f, b = work["conv21_bwd"]
    clk = mf["conv21_bwd"]["clock_mhz"]
    assert row["conv21_bwd"]["hbm_floor_ms"] == pytest.approx(b / 6.3e9, abs=1e-4)
    assert row["conv21_bwd"]["mfma_floor_ms"] == pytest.approx(f / (2.5e15 * clk / 2400) * 1e3, abs=1e-4)
    assert row["conv21_bwd"]["floor_ms"] == max(row["conv21_bwd"]["hbm_floor_ms"], row["conv21_bwd"]["mfma_floor_ms"])
    assert row["fc_dgrad"]["traffic_ratio"] == pytest.approx(tr["fc_dgrad"] / work["fc_dgrad"][1], abs=1e-3)
    # launches per step scale bytes and flops
    sr2 = step_roofline({"fc_fwd": 2.0}, {"fc_fwd": 2}, work, tr, mf, 10.0)
    assert sr2["hbm_bytes_per_step"]["pmc"] == 2 * tr["fc_fwd"]
