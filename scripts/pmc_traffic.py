"""HBM traffic per launch from rocprofv3 PMC passes (MI355X_MICROARCH.md, HBM section).

usage: python scripts/pmc_traffic.py FETCH_DIR WRITE_DIR OUT_JSON
  FETCH_DIR / WRITE_DIR: rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE --output-format csv
  output directories of the same command (separate passes: the two counters do not fit one
  TCC pass on gfx950).
Correction (gfx950): FETCH_SIZE counts half the bytes of a 16-B-per-lane streaming read
(both kernels named below read that way: LDS-DMA dwordx4 pieces), so
  traffic = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 bytes per launch.
Keys are the bench's kernel tags; values are means over that kernel's dispatches.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

# bench tag -> substring of the rocprofv3 kernel name
TAGS = {
    "vtrace": "vtrace_lds_kernel",
    "conv2_bwd": "conv2_bwd_fr",
    "conv3_bwd": "conv3_bwd_fr",
    "conv1_fwd": "conv1_fwd_fr",
    "conv1_wgrad": "conv1_wgrad_fr",
    "conv2_fwd": "conv_fwd_fr<2>",
    "conv3_fwd": "conv_fwd_fr<3>",
    "conv12_fwd": "conv12_fwd_fr",
    "conv21_bwd": "conv21_bwd_fr",
}


def read_counter(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per = defaultdict(list)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                name = row.get("Kernel_Name", "")
                per[name].append(float(row["Counter_Value"]))
    return per


def main():
    fdir, wdir, out = sys.argv[1:4]
    fetch = read_counter(fdir, "FETCH_SIZE")
    write = read_counter(wdir, "WRITE_SIZE")
    res = {}
    for tag, sub in TAGS.items():
        fk = [v for n, vs in fetch.items() if sub in n for v in vs]
        wk = [v for n, vs in write.items() if sub in n for v in vs]
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
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
