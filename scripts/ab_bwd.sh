#!/bin/bash
# A/B of the fused conv2-backward + conv1-wgrad kernel against the two separate kernels.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest -q -x tests/test_gpu_atari.py --timeout 200 > gpurun_out/ab_pytest.txt 2>&1
rc=$?; tail -3 gpurun_out/ab_pytest.txt; [ $rc -ne 0 ] && { tail -60 gpurun_out/ab_pytest.txt; exit $rc; }
for mode in fused unfused fused; do
  if [ $mode = unfused ]; then export FI_BWD_UNFUSED=1; else unset FI_BWD_UNFUSED; fi
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab_$mode.json || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/ab_$mode.json')); k=d['kernel_ms_per_step']; print('$mode', d['ms_per_step'], {x: k[x] for x in list(k)[:8]})"
done
