#!/bin/bash
# A/B of environment settings in one session: ENVS="A=1 B=1 ..." (one bench per entry, "-" = none)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
i=0
for E in ${ENVS:-- FI_BENCH_TORCH_FIRST=1 - FI_BENCH_TORCH_FIRST=1}; do
  i=$((i+1))
  if [ "$E" = "-" ]; then EV=""; else EV="$E"; fi
  env $EV timeout -k 10 200 python bench.py --steps 10 --warmup 3 --profile-steps 2 --no-cpu-baseline > gpurun_out/abe_$i.json 2>/dev/null || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/abe_$i.json')); k=d['kernel_ms_per_step']; print('$E', d['ms_per_step'], {x: k[x] for x in list(k)[:8]})"
done
