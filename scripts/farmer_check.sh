#!/bin/bash
# FarmerLstm round check: the farmer parity tests, the farmer bench line (roofline object), the
# V-trace streaming calibration probe; each step under its own time limit, stopping at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r03}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_farmer.py \
    > gpurun_out/farmer_pytest_$TAG.log 2>&1
rc=$?; echo "farmer pytest rc=$rc"; tail -3 gpurun_out/farmer_pytest_$TAG.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/farmer_bench.py --no-cpu > gpurun_out/farmer_$TAG.json 2> gpurun_out/farmer_$TAG.err
rc=$?; echo "farmer bench rc=$rc"; cat gpurun_out/farmer_$TAG.json; [ $rc -ne 0 ] && exit $rc
if [ -x build/stream_probe ]; then
  timeout -k 10 120 build/stream_probe > gpurun_out/stream_probe_$TAG.txt 2>&1
  rc=$?; echo "stream probe rc=$rc"; cat gpurun_out/stream_probe_$TAG.txt; [ $rc -ne 0 ] && exit $rc
fi
exit 0
