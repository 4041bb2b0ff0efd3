"""MFMA utilisation per kernel from one rocprofv3 pass (MI355X_MICROARCH.md: SQ_VALU_MFMA_BUSY_CYCLES
counts matrix-pipe cycles summed over SIMDs; GRBM_GUI_ACTIVE is summed over the 8 XCDs, so
GRBM_GUI_ACTIVE / 8 is the kernel's span in shader clocks and / 8 / duration its clock).

  util  = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs * GRBM_GUI_ACTIVE / 8)
  clock = GRBM_GUI_ACTIVE / 8 / kernel duration (kernel trace)

Kernels are told apart as in scripts/pmc_traffic.py: (name substring, period, phase) over one
kernel name's dispatches in dispatch order (the two MLP layers run the same GEMM instance).

usage: python scripts/pmc_mfma.py PMC_DIR OUT_JSON   (FI_BENCH_ARCH = atari | mlp)
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from freeimpala_amd import build_info  # noqa: E402

TAGS = {
    "atari": {
        "conv21_bwd": ("conv21_bwd_fr", 1, 0), "conv12_fwd": ("conv12_fwd_fr", 1, 0),
        "conv3_bwd": ("conv3_bwd_fr", 1, 0), "conv3_fwd": ("conv_fwd_fr<3>", 1, 0),
        "vtrace": ("vtrace_lds_kernel", 1, 0), "fc_wgrad": ("fc_tn_kernel", 1, 0),
        "fc_fwd": ("fcg::EpiFwd", 1, 0), "fc_dgrad": ("fcg::EpiDgrad", 1, 0),
        "heads_fwd": ("EpiHeads", 1, 0), "heads_dgrad": ("heads_dgrad", 1, 0),
        "heads_wgrad": ("heads_wgrad", 1, 0),
    },
    "mlp": {
        "vtrace": ("vtrace_lds_kernel", 1, 0),
        "mlp_fwd_l1": ("EpiBiasRelu", 2, 0), "mlp_fwd_l2": ("EpiBiasRelu", 2, 1),
        "mlp_fwd_heads": ("EpiHeads", 1, 0), "mlp_heads_bwd": ("heads_bwd_fused_f32", 1, 0),
        "mlp_wgrad_l2": ("EpiSlab", 2, 0), "mlp_wgrad_l1": ("EpiSlab", 2, 1),
        "mlp_dgrad_l2": ("EpiMask", 1, 0),
    },
}


def read_rows(d, pattern):
    files = glob.glob(os.path.join(d, "**", pattern), recursive=True)
    rows = []
    for f in files:
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    return rows


def pick(per, sub, period, phase):
    """values of every kernel name containing `sub`, every `period`-th dispatch from `phase`"""
    vals = []
    for n, vs in per.items():
        if sub in n:
            vs = sorted(vs)
            vals += [v for j, (_, v) in enumerate(vs) if j % period == phase]
    return vals


def main():
    d, out = sys.argv[1:3]
    arch = os.environ.get("FI_BENCH_ARCH", "atari")
    per = defaultdict(lambda: defaultdict(list))  # counter -> kernel name -> [(dispatch, value)]
    for i, r in enumerate(read_rows(d, "*counter_collection.csv")):
        did = int(r.get("Dispatch_Id") or r.get("Correlation_Id") or i)
        per[r["Counter_Name"]][r["Kernel_Name"]].append((did, float(r["Counter_Value"])))
    dur = defaultdict(list)
    for i, r in enumerate(read_rows(d, "*kernel_trace.csv")):
        did = int(r.get("Dispatch_Id") or r.get("Correlation_Id") or i)
        dur[r["Kernel_Name"]].append((did, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9))
    res = {}
    for tag, (sub, period, phase) in TAGS[arch].items():
        busy = pick(per["SQ_VALU_MFMA_BUSY_CYCLES"], sub, period, phase)
        act = pick(per["GRBM_GUI_ACTIVE"], sub, period, phase)
        if not busy or not act:
            continue
        b, a = sum(busy) / len(busy), sum(act) / len(act)
        e = {"dispatches": len(busy), "mfma_busy_cycles": b, "grbm_gui_active": a,
             "mfma_util": round(b / (1024 * a / 8), 4)}
        ts = pick(dur, sub, period, phase)
        if ts:
            t = sum(ts) / len(ts)
            e["duration_ms"] = round(t * 1e3, 4)
            if t >= 0.3e-3:  # the GRBM clock estimate reads high on shorter dispatches
                e["clock_mhz"] = round(a / 8 / t / 1e6, 1)
        res[tag] = e
    res["_build"] = build_info.stamp({"arch": arch})
    res["_method"] = __doc__.strip().splitlines()[0] + " -- util = SQ_VALU_MFMA_BUSY_CYCLES / (1024 * GRBM_GUI_ACTIVE / 8)"
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
