#!/bin/bash
# gpu_tests.sh TAG [pytest targets...] -- one gpurun step: the named GPU tests (default: all),
# then optionally the farmer bench (FARMER=1) and the learner bench (BENCH=atari|mlp). Each
# GPU step has its own time limit; a failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
TAG=$1
shift
TARGETS=${*:-tests}
timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest -x -v ${PYTEST_ARGS:-} --timeout 120 --timeout-method thread -m gpu $TARGETS \
    > "$OUT/pytest_$TAG.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 "$OUT/pytest_$TAG.log"
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" "$OUT/pytest_$TAG.log" | head -20; exit $rc; }
if [ "${FARMER:-0}" = 1 ]; then
  timeout -k 10 300 python scripts/farmer_bench.py ${FARMER_ARGS:-} > "$OUT/farmer_$TAG.json" 2> "$OUT/farmer_$TAG.err"
  rc=$?; echo "farmer rc=$rc"; cat "$OUT/farmer_$TAG.json"; [ $rc -ne 0 ] && { tail -5 "$OUT/farmer_$TAG.err"; exit $rc; }
fi
if [ -n "${BENCH:-}" ]; then
  timeout -k 10 600 python bench.py --arch "$BENCH" ${BENCH_ARGS:-} > "$OUT/bench_${BENCH}_$TAG.json" 2> "$OUT/bench_${BENCH}_$TAG.err"
  rc=$?; echo "bench rc=$rc"; cat "$OUT/bench_${BENCH}_$TAG.json"; [ $rc -ne 0 ] && { tail -5 "$OUT/bench_${BENCH}_$TAG.err"; exit $rc; }
fi
exit 0
