#!/bin/bash
# A/B of experiment libraries (build/ab/lib_NAME.so) on the Atari bench: ms/step and the
# three largest conv kernels, interleaved with the default library to see box drift.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {
  local n=$1
  if [ "$n" = default ]; then unset FI_LIB_OVERRIDE; else export FI_LIB_OVERRIDE=build/ab/lib_$n.so; fi
  timeout -k 10 200 python bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline > gpurun_out/ab_$n.json 2> gpurun_out/ab_$n.err || { echo "FAIL $n"; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab_$n.json')); k=d['kernel_ms_per_step']; print('$n', round(d['ms_per_step'],3), {x: k[x] for x in ('conv21_bwd','conv12_fwd','conv3_bwd','conv3_fwd')})"
}
for n in default ${LIBS}; do run $n; done
run default
