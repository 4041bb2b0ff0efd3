#!/bin/bash
# vt_rocprof.sh TAG -- rocprofv3 kernel-trace summaries of the stand-alone V-trace kernel 1,
# cold (6 rotating input/output sets) and warm (one set), so its kernel duration (no dispatch
# gap between back-to-back launches) can be set beside bench.py's event-based figure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; TAG=${1:-r03}
mkdir -p "$OUT"; export TMPDIR=/tmp; cd /tmp
for S in 6 1; do
  rm -rf "$OUT/vtprof_s${S}_$TAG"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/vtprof_s${S}_$TAG" -o run \
      -- python3 "$ROOT/scripts/vtrace_bench.py" --variant 1 --sets $S --iters 100 > "$OUT/vtprof_s${S}_$TAG.log" 2>&1
  rc=$?; echo "sets $S rc=$rc"; cat "$OUT/vtprof_s${S}_$TAG.log"; [ $rc -ne 0 ] && exit $rc
done
exit 0
