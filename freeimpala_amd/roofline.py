"""Step-level roofline of the learner step (bench.py's `step_roofline` field).

The per-kernel roofline of bench.py's line prices one kernel; this prices the whole step:
  * HBM bytes per step = the stamped rocprofv3 PMC traffic (FETCH_SIZE x 2 + WRITE_SIZE, per
    launch, MI355X_MICROARCH.md's gfx950 correction) x the launches per step, summed over every
    kernel of the step; a kernel the counter pass has no entry for is counted at its
    algorithmic bytes and named;
  * achieved TB/s = those bytes / the timed ms_per_step, as a fraction of the 8 TB/s spec peak
    and of the ~6.3 TB/s a streaming kernel reaches on MI355X;
  * MFMA floor = the dense bf16 FLOPs / 2.5 PF/s, and at each kernel's PMC clock
    (2.5 PF/s x clock / 2400 MHz);
  * per kernel: its time in the profiled pass, its floor max(HBM, MFMA) and the gap between,
    sorted by gap -- the next target is the largest gap, not the largest share.
Pure arithmetic over plain dicts: tests/test_step_roofline.py checks it against the stamped file.
"""
from __future__ import annotations

HBM_PEAK_TBS = 8.0          # MI355X HBM3E spec
HBM_ACHIEVABLE_TBS = 6.3    # MI355X_MICROARCH.md: achievable streaming bandwidth
MFMA_PEAK_TFLOPS = {"bf16": 2500.0, "fp32": 157.3}
PEAK_CLOCK_MHZ = 2400.0


def step_roofline(kernel_ms: dict, launches: dict, work: dict, traffic: dict, mfma: dict,
                  ms_per_step: float, dtype: str = "bf16") -> dict:
    """kernel_ms[k]: ms per step of kernel k (profiled pass); launches[k]: launches per step;
    work[k]: (flops, bytes) algorithmic per launch; traffic[k]: PMC HBM bytes per launch;
    mfma[k]: {"clock_mhz": ...} from the stamped MFMA pass; ms_per_step: the timed loop's."""
    peak_f = MFMA_PEAK_TFLOPS[dtype] * 1e12
    pmc_bytes = alg_bytes = flops_total = 0.0
    mfma_ms_clock = 0.0
    no_pmc, unmodelled, rows = [], [], []
    for k, ms in kernel_ms.items():
        n = launches.get(k, 1)
        if k not in work:
            unmodelled.append(k)
            rows.append({"kernel": k, "ms": round(ms, 4), "floor_ms": None, "gap_ms": round(ms, 4)})
            continue
        f, b = work[k]
        f, b = f * n, b * n
        tr = traffic.get(k)
        moved = tr * n if tr is not None else b
        if tr is None:
            no_pmc.append(k)
        pmc_bytes += moved
        alg_bytes += b
        flops_total += f
        clk = (mfma.get(k) or {}).get("clock_mhz") or PEAK_CLOCK_MHZ
        t_mfma = f / (peak_f * clk / PEAK_CLOCK_MHZ) * 1e3
        mfma_ms_clock += t_mfma
        t_hbm = b / (HBM_ACHIEVABLE_TBS * 1e12) * 1e3
        floor = max(t_hbm, t_mfma)
        rows.append({"kernel": k, "ms": round(ms, 4), "launches": n,
                     "hbm_floor_ms": round(t_hbm, 4), "mfma_floor_ms": round(t_mfma, 4),
                     "bound": "hbm" if t_hbm >= t_mfma else "mfma",
                     "floor_ms": round(floor, 4), "gap_ms": round(ms - floor, 4),
                     "traffic_ratio": round(moved / b, 3) if b else None})
    rows.sort(key=lambda r: -r["gap_ms"])
    floor_sum = sum(r["floor_ms"] for r in rows if r["floor_ms"] is not None)
    tbs = pmc_bytes / (ms_per_step * 1e-3) / 1e12
    return {
        "hbm_bytes_per_step": {"pmc": int(pmc_bytes), "algorithmic": int(alg_bytes),
                               "kernels_at_algorithmic_bytes": sorted(no_pmc)},
        "ms_per_step": round(ms_per_step, 4),
        "achieved_tbs": round(tbs, 3),
        "frac_of_peak_8tbs": round(tbs / HBM_PEAK_TBS, 4),
        "frac_of_achievable_6p3tbs": round(tbs / HBM_ACHIEVABLE_TBS, 4),
        "hbm_floor_ms": {"pmc_bytes_at_6p3tbs": round(pmc_bytes / (HBM_ACHIEVABLE_TBS * 1e9), 3),
                         "pmc_bytes_at_8tbs": round(pmc_bytes / (HBM_PEAK_TBS * 1e9), 3),
                         "algorithmic_at_6p3tbs": round(alg_bytes / (HBM_ACHIEVABLE_TBS * 1e9), 3)},
        "mfma_floor_ms": {"at_2400mhz": round(flops_total / peak_f * 1e3, 3),
                          "at_pmc_clocks": round(mfma_ms_clock, 3)},
        "sum_of_kernel_floors_ms": round(floor_sum, 3),
        "frac_of_kernel_floors": round(floor_sum / ms_per_step, 4),
        "unmodelled_kernels": sorted(unmodelled),
        "kernels_by_gap": rows,
        "method": ("kernel ms from the profiled pass (HIP events per launch after the timed loop); "
                   "per-kernel floor = max(algorithmic bytes / 6.3 TB/s, dense FLOPs / (2.5 PF/s x PMC "
                   "clock / 2400 MHz)); gap = ms - floor; achieved = PMC bytes / timed ms_per_step"),
    }
