#!/bin/bash
# ab_libs.sh LIB... -- one short bench per library ("" = the product library), top kernels
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for L in "$@"; do
  [ "$L" = prod ] && L=""
  FI_LIB_OVERRIDE=$L timeout -k 10 200 python bench.py --steps 8 --warmup 3 --sustain-seconds 0 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab.json 2>gpurun_out/ab.err || exit 1
  python3 -c "
import json, os; d=json.load(open('gpurun_out/ab.json')); k=d['kernel_ms_per_step']; sel=os.environ.get('AB_KERNELS'); print('${L:-prod}', round(d['ms_per_step'],3), {x: k[x] for x in (sel.split(',') if sel else list(k)[:7]) if x in k})"
done
