#!/bin/bash
# ab_r04.sh -- round-4 GPU step: farmer + conv21 parity tests, the farmer bench fused / unfused,
# then interleaved Atari A/B of the build/ab variant libraries (scripts/build_exp.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_farmer.py \
    tests/test_gpu_atari.py -k "${TESTK:-farmer or fused_conv21 or production_path}" > gpurun_out/pytest_${TAG:-r04c}.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_${TAG:-r04c}.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/pytest_${TAG:-r04c}.log | head; exit $rc; }
for m in fused unfused; do
  if [ $m = unfused ]; then export FI_FARMER_UNFUSED=1; else unset FI_FARMER_UNFUSED; fi
  timeout -k 10 300 python scripts/farmer_bench.py --configs 32x10,512x100 --no-cpu > gpurun_out/farmer_${m}.json 2> gpurun_out/farmer_${m}.err
  rc=$?; echo "farmer $m rc=$rc"; grep -o '"B": [0-9]*\|"ms_per_step": [0-9.]*\|"value": [0-9.]*' gpurun_out/farmer_${m}.json | tr '\n' ' '; echo
  [ $rc -ne 0 ] && { tail -5 gpurun_out/farmer_${m}.err; exit $rc; }
done
unset FI_FARMER_UNFUSED
for r in 1 2; do
  bash scripts/ab_libs.sh ${LIBS:-prod} || exit 1
done
exit 0
