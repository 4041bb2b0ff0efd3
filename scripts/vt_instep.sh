#!/bin/bash
# V-trace load-policy A/B: each build/ab/lib_vt_<v>.so (VT_LIBS) timed stand-alone cold / warm
# (scripts/vtrace_bench.py) and inside the Atari learner step (bench.py through FI_LIB_OVERRIDE:
# kernel_ms_per_step.vtrace, the in-step event time).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r03}
mkdir -p gpurun_out
L=""
for v in ${VT_LIBS:-plain munt allnt plain}; do L="$L --lib build/ab/lib_vt_$v.so"; done
timeout -k 10 240 python scripts/vtrace_bench.py $L --variant 1 --sets 6 > gpurun_out/vti_cold_$TAG.txt 2>&1 || exit $?
timeout -k 10 240 python scripts/vtrace_bench.py $L --variant 1 --sets 1 > gpurun_out/vti_warm_$TAG.txt 2>&1 || exit $?
cat gpurun_out/vti_cold_$TAG.txt gpurun_out/vti_warm_$TAG.txt
for v in ${VT_LIBS:-plain munt allnt plain}; do
  FI_LIB_OVERRIDE=build/ab/lib_vt_$v.so timeout -k 10 300 python bench.py --arch ${ARCH:-atari} --no-cpu-baseline \
      > gpurun_out/vti_bench_${v}_$TAG.json 2> gpurun_out/vti_bench_${v}_$TAG.err || exit $?
  python -c "
import json,sys
d=json.loads(open('gpurun_out/vti_bench_${v}_$TAG.json').read().strip().splitlines()[-1])
print('$v', 'step_ms', d['ms_per_step'], 'vtrace in-step ms', d['kernel_ms_per_step']['vtrace'], 'event', d['roofline_vtrace']['in_step_event_ms'], 'cold', d['roofline_vtrace']['launch_ms'], 'warm', d['roofline_vtrace']['warm']['launch_ms'])"
done
