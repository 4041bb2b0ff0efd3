"""MFMA utilisation per kernel from one rocprofv3 pass (MI355X_MICROARCH.md: SQ_VALU_MFMA_BUSY_CYCLES
counts matrix-pipe cycles summed over SIMDs; GRBM_GUI_ACTIVE is summed over the 8 XCDs, so
GRBM_GUI_ACTIVE / 8 is the kernel's span in shader clocks and / 8 / duration its clock).

  util  = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs * GRBM_GUI_ACTIVE / 8)
  clock = GRBM_GUI_ACTIVE / 8 / kernel duration (kernel trace)

usage: python scripts/pmc_mfma.py PMC_DIR OUT_JSON
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from freeimpala_amd import build_info  # noqa: E402

TAGS = {"conv21_bwd": "conv21_bwd_fr", "conv12_fwd": "conv12_fwd_fr", "conv3_bwd": "conv3_bwd_fr",
        "conv3_fwd": "conv_fwd_fr<3>", "vtrace": "vtrace_lds_kernel", "fc_wgrad": "fc_tn_kernel",
        "fc_nt (own fwd/dgrad)": "fc_nt_kernel", "fc (hipBLASLt)": "Cijk_",
        # MLP (config #2 network): the dominant kernel of that line is the data gradient of layer 2
        "mlp_dgrad_l2": "EpiMask", "mlp_heads_bwd": "heads_bwd_fused_f32", "mlp_fwd_heads": "EpiHeads"}


def main():
    d, out = sys.argv[1:3]
    cnt = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            for tag, sub in TAGS.items():
                if sub in r["Kernel_Name"]:
                    cnt[tag][r["Counter_Name"]].append(float(r["Counter_Value"]))
    dur = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            for tag, sub in TAGS.items():
                if sub in r["Kernel_Name"]:
                    dur[tag].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    res = {}
    for tag, cs in cnt.items():
        busy = cs.get("SQ_VALU_MFMA_BUSY_CYCLES", [])
        act = cs.get("GRBM_GUI_ACTIVE", [])
        if not busy or not act:
            continue
        b, a = sum(busy) / len(busy), sum(act) / len(act)
        e = {"dispatches": len(busy), "mfma_busy_cycles": b, "grbm_gui_active": a,
             "mfma_util": round(b / (1024 * a / 8), 4)}
        if dur.get(tag):
            t = sum(dur[tag]) / len(dur[tag])
            e["duration_ms"] = round(t * 1e3, 4)
            if t >= 0.3e-3:  # the GRBM clock estimate reads high on shorter dispatches
                e["clock_mhz"] = round(a / 8 / t / 1e6, 1)
        res[tag] = e
    res["_build"] = build_info.stamp({"arch": os.environ.get("FI_BENCH_ARCH", "atari")})
    res["_method"] = __doc__.strip().splitlines()[0] + " -- util = SQ_VALU_MFMA_BUSY_CYCLES / (1024 * GRBM_GUI_ACTIVE / 8)"
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
