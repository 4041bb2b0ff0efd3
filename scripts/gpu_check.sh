#!/bin/bash
# One gpurun session: GPU parity tests, bench, rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a fault / abort / timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
ARCH=${ARCH:-mlp}
TAG=${TAG:-r01}
fatal() { case $1 in 0|1) return 1;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }

if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest tests -v -m gpu ${PYTEST_ARGS:--x} --timeout=300 --timeout-method thread \
      > "$OUT/pytest_gpu_$TAG.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 "$OUT/pytest_gpu_$TAG.log"
  fatal $rc pytest || true
fi
timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py --arch "$ARCH" ${BENCH_ARGS:-} \
    > "$OUT/bench_${ARCH}_$TAG.json" 2> "$OUT/bench_${ARCH}_$TAG.err"
rc=$?; echo "bench rc=$rc"; cat "$OUT/bench_${ARCH}_$TAG.json"; tail -3 "$OUT/bench_${ARCH}_$TAG.err"
[ $rc -ne 0 ] && exit $rc
if [ "${SKIP_PROF:-0}" != 1 ]; then
  export TMPDIR=/tmp
  cd /tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_${ARCH}_$TAG" -o run \
      -- python3 "$ROOT/bench.py" --arch "$ARCH" --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} \
      > "$OUT/prof_${ARCH}_$TAG.log" 2>&1
  rc=$?; echo "rocprof rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  find "$OUT/prof_${ARCH}_$TAG" -name "*kernel_stats.csv" | head -3
fi
exit 0
