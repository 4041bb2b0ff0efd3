#!/bin/bash
# quick GPU iteration: atari parity tests, a stamps build (if present), a short bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 300 python -m pytest -q -x tests/test_gpu_atari.py 2>&1 | tail -1 || exit 1
if [ -f build/exp/lib_st.so ]; then
  FI_LIB_OVERRIDE=build/exp/lib_st.so timeout -k 10 200 python bench.py --steps 2 --warmup 1 --profile-steps 1 --no-cpu-baseline > /dev/null || exit 1
fi
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/b.json || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/b.json')); print(d['ms_per_step'], d['kernel_ms_per_step'])"
