#!/bin/bash
# vt_r04.sh TAG -- the streaming V-trace kernel (variant 4) against the chunked kernel (1):
# parity tests, cold / warm replay timings interleaved, rocprofv3 kernel durations of both cold.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; TAG=${1:-r04}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_vtrace.py > "$OUT/pytest_vt_$TAG.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/pytest_vt_$TAG.log"; [ $rc -ne 0 ] && { grep -E "FAILED|Error" "$OUT/pytest_vt_$TAG.log" | head; exit $rc; }
for r in 1 2; do
  for S in 6 1; do
    timeout -k 10 200 python scripts/vtrace_bench.py --variant 1 --variant 4 --sets $S --iters 100 > "$OUT/vtbench_s${S}_${r}_$TAG.txt" 2>&1
    rc=$?; echo "bench sets=$S round $r rc=$rc"; cat "$OUT/vtbench_s${S}_${r}_$TAG.txt"; [ $rc -ne 0 ] && exit $rc
  done
done
export TMPDIR=/tmp; cd /tmp
for V in 4 1; do
  rm -rf "$OUT/vtprof_v${V}_$TAG"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/vtprof_v${V}_$TAG" -o run \
      -- python3 "$ROOT/scripts/vtrace_bench.py" --variant $V --sets 6 --iters 100 > "$OUT/vtprof_v${V}_$TAG.log" 2>&1
  rc=$?; echo "rocprof v$V rc=$rc"; [ $rc -ne 0 ] && exit $rc
  find "$OUT/vtprof_v${V}_$TAG" -name "*kernel_stats.csv" -exec grep -h "vtrace" {} \; | cut -c1-200
done
exit 0
