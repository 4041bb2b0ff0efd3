#!/usr/bin/env python3
"""design_tables.py BENCH_JSON [PMC_TRAFFIC_JSON PMC_MFMA_JSON] -- DESIGN.md section 5's per-kernel
table from a bench line (its step_roofline, i.e. the profiled pass's kernel ms) and the stamped
counter summaries: ms, floor, gap, bound, PMC traffic / algorithmic bytes, MFMA busy and clock.
Every number in the table is read from the files named on the command line."""
import json
import sys


def load(p):
    with open(p) as fh:
        txt = fh.read().strip()
    return json.loads(txt.splitlines()[-1] if not txt.startswith("{\n") else txt)


def main():
    b = load(sys.argv[1])
    tr = {k: v for k, v in load(sys.argv[2]).items() if not k.startswith("_")} if len(sys.argv) > 2 else {}
    mf = {k: v for k, v in load(sys.argv[3]).items() if not k.startswith("_")} if len(sys.argv) > 3 else {}
    sr = b["step_roofline"]
    print(f"step: {b['ms_per_step']} ms timed; PMC bytes {sr['hbm_bytes_per_step']['pmc'] / 1e9:.2f} GB "
          f"(algorithmic {sr['hbm_bytes_per_step']['algorithmic'] / 1e9:.2f} GB) -> {sr['achieved_tbs']} TB/s = "
          f"{sr['frac_of_peak_8tbs']} of 8 TB/s, {sr['frac_of_achievable_6p3tbs']} of 6.3 TB/s; "
          f"HBM floor {sr['hbm_floor_ms']}; MFMA floor {sr['mfma_floor_ms']}; sum of kernel floors "
          f"{sr['sum_of_kernel_floors_ms']} ms ({sr['frac_of_kernel_floors']} of the step)")
    print()
    print("| kernel | ms | floor ms (bound) | gap ms | PMC traffic ÷ algorithmic | MFMA busy @ MHz |")
    print("|---|---|---|---|---|---|")
    for r in sr["kernels_by_gap"]:
        k = r["kernel"]
        m = mf.get(k, {})
        busy = f"{m['mfma_util']:.2f} @ {m['clock_mhz']:.0f}" if m.get("clock_mhz") and m.get("mfma_util") else "—"
        if r["floor_ms"] is None:
            print(f"| {k} | {r['ms']:.3f} | — | {r['gap_ms']:.3f} | — | — |")
            continue
        t = tr.get(k, {}).get("hbm_bytes_per_launch")
        ratio = f"{r['traffic_ratio']:.2f}×" if t is not None and r.get("traffic_ratio") else "—"
        print(f"| {k} | {r['ms']:.3f} | {r['floor_ms']:.3f} ({r['bound']}) | {r['gap_ms']:.3f} | {ratio} | {busy} |")


if __name__ == "__main__":
    main()
