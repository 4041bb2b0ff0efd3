"""Build identity of libfi_learner.so's sources, used to stamp counter passes.

`source_hash()` is a sha256 over every file the learner step's kernels are built from
(freeimpala_amd/csrc/* except the FarmerLstm step's farmer.hip, include/fi_learner.h, the
Makefile; the learner never launches a farmer kernel), so a rocprofv3 PMC summary under
profiles/ can be matched to the exact kernels a bench line timed: bench.py attaches counter
fields (HBM traffic, MFMA utilisation) only from a summary whose `_build.source_hash` equals the
hash of the tree it runs from, and reports them as null otherwise.
"""
from __future__ import annotations

import glob
import hashlib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def source_files():
    files = sorted(glob.glob(os.path.join(ROOT, "freeimpala_amd", "csrc", "*")))
    files = [f for f in files if os.path.basename(f) != "farmer.hip"]
    files += [os.path.join(ROOT, p) for p in ("include/fi_learner.h", "Makefile")]
    return [f for f in files if os.path.isfile(f)]


def source_hash() -> str:
    h = hashlib.sha256()
    for f in source_files():
        h.update(os.path.relpath(f, ROOT).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()[:16]


# run-time switches that change which kernels the learner step launches, or how: a counter pass
# taken under one setting says nothing about a bench line timed under another
KERNEL_ENV = ("FI_FR_GRID", "FI_KEEP_DA1", "FI_BWD_UNFUSED", "FI_FWD_UNFUSED",
              "FI_A1_NHWC", "FI_ATARI_GENERIC")


def rocm_version() -> str:
    for p in ("/opt/rocm/.info/version", "/opt/rocm/.info/version-dev"):
        try:
            with open(p) as fh:
                return fh.read().strip()
        except OSError:
            pass
    return "unknown"


def runtime_key() -> dict:
    """The kernel-relevant FI_* environment (set ones only) and the ROCm release."""
    return {"env": {k: os.environ[k] for k in KERNEL_ENV if k in os.environ}, "rocm": rocm_version()}


def stamp(extra=None) -> dict:
    """The `_build` object a counter summary carries."""
    d = {"source_hash": source_hash(), "runtime": runtime_key()}
    if extra:
        d.update(extra)
    return d


if __name__ == "__main__":
    print(source_hash())
