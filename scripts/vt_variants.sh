#!/bin/bash
# V-trace kernel-1 A/B: every build/ab/lib_vt_*.so named in VT_LIBS timed cold (6 rotating sets)
# and warm through scripts/vtrace_bench.py, base library first and last.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r03}
mkdir -p gpurun_out
L="--lib build/ab/lib_vt_base.so"
for v in ${VT_LIBS:-nt ldnt ldsc1 ldsc0sc1 nw2 nw2nt}; do L="$L --lib build/ab/lib_vt_$v.so"; done
L="$L --lib build/ab/lib_vt_base.so"
timeout -k 10 240 python scripts/vtrace_bench.py $L --variant 1 --sets 6 > gpurun_out/vt_cold_$TAG.txt 2>&1 || exit $?
timeout -k 10 240 python scripts/vtrace_bench.py $L --variant 1 --sets 1 > gpurun_out/vt_warm_$TAG.txt 2>&1 || exit $?
cat gpurun_out/vt_cold_$TAG.txt gpurun_out/vt_warm_$TAG.txt
