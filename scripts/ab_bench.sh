#!/bin/bash
# ab_bench.sh TAG LIB... -- the Atari bench line (no CPU baseline) once per experiment library
# (FI_LIB_OVERRIDE), interleaved twice; prints step ms and the per-kernel times that differ.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
mkdir -p gpurun_out
for rep in 1 2; do
  for L in "$@"; do
    n=$(basename $L .so)
    FI_LIB_OVERRIDE=$L timeout -k 10 300 python bench.py --arch ${ARCH:-atari} --no-cpu-baseline --steps 20 \
        > gpurun_out/ab_${TAG}_${n}_$rep.json 2> gpurun_out/ab_${TAG}_${n}_$rep.err || exit $?
    python -c "
import json
d=json.loads(open('gpurun_out/ab_${TAG}_${n}_$rep.json').read().strip().splitlines()[-1])
k=d['kernel_ms_per_step']
print('$n rep $rep', 'step', d['ms_per_step'], {x: k[x] for x in list(k)[:6]})"
  done
done
