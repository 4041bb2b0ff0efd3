#!/bin/bash
# round_check.sh TAG -- one gpurun call: every GPU test, smoke(), the Atari and MLP bench lines
# and a rocprofv3 kernel-trace summary of each bench. Each GPU step under its own time limit;
# the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
TAG=${1:-r03}
mkdir -p "$OUT"
# long silent steps (the full-size fp64 gradient check, the whole-step CPU baseline): a heartbeat
# file under gpurun_out shows the call is alive
( while sleep 30; do date +%T >> "$OUT/heartbeat_$TAG.txt"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export FI_TEST_REPORT_DIR=$OUT
timeout -k 10 900 python -u -m pytest tests -v -m gpu -x --timeout 120 --timeout-method thread > "$OUT/pytest_gpu_$TAG.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest_gpu_$TAG.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.txt" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 "$OUT/smoke_$TAG.txt"; [ $rc -ne 0 ] && exit $rc
for A in atari mlp; do
  timeout -k 10 400 python bench.py --arch $A > "$OUT/bench_${A}_$TAG.json" 2> "$OUT/bench_${A}_$TAG.err"
  rc=$?; echo "bench $A rc=$rc"; cat "$OUT/bench_${A}_$TAG.json"; [ $rc -ne 0 ] && { tail -5 "$OUT/bench_${A}_$TAG.err"; exit $rc; }
done
export TMPDIR=/tmp
cd /tmp
for A in atari mlp; do
  rm -rf "$OUT/prof_${A}_$TAG"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_${A}_$TAG" -o run \
      -- python3 "$ROOT/bench.py" --arch $A --steps 5 --warmup 2 --sustain-seconds 0 --no-cpu-baseline > "$OUT/prof_${A}_$TAG.log" 2>&1
  rc=$?; echo "rocprof $A rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
