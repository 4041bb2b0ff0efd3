#!/bin/bash
# per-phase clocks + per-kernel ms of several FI_PHASES experiment builds (build/exp/lib_NAME.so)
# (the instrumentation lives in scripts/patches/atari_fr_phase_clocks.patch: apply it first)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for L in ${LIBS:-ph}; do
  FI_LIB_OVERRIDE=build/ab/lib_$L.so timeout -k 10 200 python bench.py --steps 3 --warmup 2 --profile-steps 1 --no-cpu-baseline > gpurun_out/ph_$L.json 2> gpurun_out/ph_$L.txt || exit 1
  echo "== $L $(python3 -c "import json; d=json.load(open('gpurun_out/ph_$L.json')); k=d['kernel_ms_per_step']; print(d['ms_per_step'], {x: k[x] for x in list(k)[:3]})")"
  grep "phases ${PH_KERNEL:-conv21}" gpurun_out/ph_$L.txt
done
