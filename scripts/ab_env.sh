#!/bin/bash
# ab_env.sh ROUNDS "ENV_A" "ENV_B" ... -- interleaved A/B of run-time switches on one box: each
# round runs one bench per setting ("-" = no extra environment), printing ms/step and the
# profiled pass's top kernels. Every bench under its own time limit; a failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$1; shift
mkdir -p gpurun_out
for r in $(seq 1 "$R"); do
  for E in "$@"; do
    [ "$E" = - ] && E=""
    env $E timeout -k 10 200 python bench.py --steps ${STEPS:-30} --warmup 5 --sustain-seconds 0 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/abe.json 2>gpurun_out/abe.err || { tail -5 gpurun_out/abe.err; exit 1; }
    python3 -c "
import json, os; d=json.load(open('gpurun_out/abe.json')); k=d['kernel_ms_per_step']; p=d['phase_ms']; sel=os.environ.get('AB_KERNELS')
print('r$r', '${E:-default}', round(d['ms_per_step'],3), 'bwd', round(p['backward'],3), {x: k[x] for x in (sel.split(',') if sel else list(k)[:8]) if x in k})"
  done
done
