"""Summarise the pmc_instmix.sh passes: per kernel, the mean of each counter over its launches,
plus derived per-wave ratios. usage: pmc_instmix.py OUTDIR SUMMARY.json"""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from freeimpala_amd import build_info  # noqa: E402

KERNELS = ["conv21_bwd_fr", "conv3_bwd_fr", "conv12_fwd_fr", "conv_fwd_fr<3>", "vtrace_lds_kernel",
           "heads_dgrad", "heads_wgrad"]


def main(outdir, dst):
    d = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(f"{outdir}/pmcmix_*/**/*counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            for k in KERNELS:
                if k in n:
                    d[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {}
    for k, cs in d.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        out = {"counters": {c: round(v, 1) for c, v in sorted(m.items())}}
        waves = m.get("SQ_WAVES")
        if waves:
            out["per_wave"] = {c: round(m[c] / waves, 1) for c in
                               ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_INSTS_SALU",
                                "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR") if c in m}
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            out["frac_of_wave_cycles"] = {c: round(m[c] / wc, 3) for c in
                                          ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS",
                                           "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                                           "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_MISC") if c in m}
        if "SQ_LDS_BANK_CONFLICT" in m and "SQ_LDS_IDX_ACTIVE" in m and m["SQ_LDS_IDX_ACTIVE"]:
            out["lds_bank_conflict_per_active"] = round(m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"], 4)
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m and m["GRBM_GUI_ACTIVE"]:
            # util = busy / (SIMDs x GRBM_GUI_ACTIVE / 8 XCDs), as scripts/pmc_mfma.py
            out["mfma_util"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * m["GRBM_GUI_ACTIVE"] / 8), 4)
        res[k] = out
    res["_build"] = build_info.stamp({"arch": os.environ.get("FI_BENCH_ARCH", "atari")})
    with open(dst, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
