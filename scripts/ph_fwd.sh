#!/bin/bash
# per-phase clocks of the frame-resident kernels (FI_PHASES build) -> gpurun_out/ph.txt
# (the instrumentation lives in scripts/patches/atari_fr_phase_clocks.patch: apply it first)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
FI_LIB_OVERRIDE=build/exp/lib_${PH_LIB:-ph}.so timeout -k 10 200 python bench.py --steps 3 --warmup 2 --profile-steps 1 --no-cpu-baseline > gpurun_out/ph.json 2> gpurun_out/ph.txt || exit 1
grep phases gpurun_out/ph.txt
