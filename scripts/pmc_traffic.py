"""HBM traffic per launch from rocprofv3 PMC passes (MI355X_MICROARCH.md, HBM section).

usage: python scripts/pmc_traffic.py FETCH_DIR WRITE_DIR OUT_JSON [ARCH]
  FETCH_DIR / WRITE_DIR: rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE --output-format csv
  output directories of the same command (separate passes: the two counters do not fit one
  TCC pass on gfx950). ARCH: atari (default) or mlp -- which bench tags to summarise.
Correction (gfx950): FETCH_SIZE counts half the bytes of a 16-B-per-lane streaming read
(the kernels here read that way: LDS-DMA / dwordx4 pieces), so
  traffic = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 bytes per launch.
Keys are the bench's kernel tags; values are means over that kernel's dispatches. A tag whose
kernel is launched several times per step under one name (the MLP's fp32 GEMM instances) is
picked by its position in the step: (substring, period, phase) over the dispatches of that
name in dispatch order. The summary is stamped with freeimpala_amd.build_info.stamp() so
bench.py only attaches it to a line timed on the same sources.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from freeimpala_amd import build_info  # noqa: E402

# bench tag -> (substring of the rocprofv3 kernel name, dispatches of that name per step, index)
TAGS = {
    "atari": {
        "vtrace": ("vtrace_lds_kernel", 1, 0),
        "conv12_fwd": ("conv12_fwd_fr", 1, 0),
        "conv3_fwd": ("conv_fwd_fr<3>", 1, 0),
        "conv3_bwd": ("conv3_bwd_fr", 1, 0),
        "conv21_bwd": ("conv21_bwd_fr", 1, 0),
        "fc_wgrad": ("fc_tn_kernel", 1, 0),
        "fc_fwd": ("fcg::EpiFwd", 1, 0),
        "fc_dgrad": ("fcg::EpiDgrad", 1, 0),
        "heads_dgrad": ("heads_dgrad", 1, 0),
        "heads_wgrad": ("heads_wgrad", 1, 0),
        "heads_fwd": ("EpiHeads", 1, 0),
    },
    "mlp": {
        "vtrace": ("vtrace_lds_kernel", 1, 0),
        "mlp_fwd_l1": ("EpiBiasRelu", 2, 0),
        "mlp_fwd_l2": ("EpiBiasRelu", 2, 1),
        "mlp_fwd_heads": ("EpiHeads", 1, 0),
        "mlp_heads_bwd": ("heads_bwd_fused_f32", 1, 0),
        "mlp_wgrad_l2": ("EpiSlab", 2, 0),
        "mlp_wgrad_l1": ("EpiSlab", 2, 1),
        "mlp_dgrad_l2": ("EpiMask", 1, 0),
    },
}


def read_counter(d, counter):
    """kernel name -> [(dispatch id, value)] sorted by dispatch id"""
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per = defaultdict(list)
    for f in files:
        with open(f) as fh:
            for i, row in enumerate(csv.DictReader(fh)):
                if row.get("Counter_Name") != counter:
                    continue
                did = row.get("Dispatch_Id") or row.get("Correlation_Id") or i
                per[row.get("Kernel_Name", "")].append((int(did), float(row["Counter_Value"])))
    for v in per.values():
        v.sort()
    return per


def pick(per, sub, period, phase):
    vals = []
    for n, vs in per.items():
        if sub in n:
            vals += [v for j, (_, v) in enumerate(vs) if j % period == phase]
    return vals


def main():
    fdir, wdir, out = sys.argv[1:4]
    arch = sys.argv[4] if len(sys.argv) > 4 else "atari"
    fetch = read_counter(fdir, "FETCH_SIZE")
    write = read_counter(wdir, "WRITE_SIZE")
    res = {}
    for tag, (sub, period, phase) in TAGS[arch].items():
        fk, wk = pick(fetch, sub, period, phase), pick(write, sub, period, phase)
        if not fk or not wk:
            continue
        f_kb = sum(fk) / len(fk)
        w_kb = sum(wk) / len(wk)
        res[tag] = {"fetch_size_kb": round(f_kb, 1), "write_size_kb": round(w_kb, 1),
                    "dispatches": min(len(fk), len(wk)),
                    "hbm_bytes_per_launch": int((2 * f_kb + w_kb) * 1024)}
    res["_method"] = ("rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes of "
                      "the same bench command; traffic = (2*FETCH_SIZE + WRITE_SIZE) KiB per launch "
                      "(gfx950 FETCH_SIZE half-count correction)")
    res["_build"] = build_info.stamp({"arch": arch, "config": "T=100 B=4096 A=18"})
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
