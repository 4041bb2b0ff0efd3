#!/bin/bash
# A/B of experiment builds (build/exp/lib_NAME.so): short bench each, per-kernel ms.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for L in ${LIBS:-base plain base plain}; do
  FI_LIB_OVERRIDE=build/exp/lib_$L.so timeout -k 10 200 python bench.py --steps 6 --warmup 2 --profile-steps 2 --no-cpu-baseline > gpurun_out/ab_$L.json 2>/dev/null || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/ab_$L.json')); k=d['kernel_ms_per_step']; print('$L', d['ms_per_step'], {x: k[x] for x in list(k)[:7]})"
done
