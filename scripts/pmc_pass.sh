#!/bin/bash
# Two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) over a short bench run, then the per-launch
# HBM traffic summary (scripts/pmc_traffic.py). Counters only: no trace domains in these runs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
TAG=${TAG:-r01}
ARCH=${ARCH:-atari}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for C in FETCH_SIZE WRITE_SIZE; do
  rm -rf "$OUT/pmc_${C}_${ARCH}_$TAG"
  timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_${C}_${ARCH}_$TAG" -o run \
      -- python3 "$ROOT/bench.py" --arch "$ARCH" --steps 2 --warmup 1 --profile-steps 1 --sustain-seconds 0 --no-cpu-baseline \
      > "$OUT/pmc_${C}_${ARCH}_$TAG.log" 2>&1
  rc=$?; echo "pmc $C rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
python3 "$ROOT/scripts/pmc_traffic.py" "$OUT/pmc_FETCH_SIZE_${ARCH}_$TAG" "$OUT/pmc_WRITE_SIZE_${ARCH}_$TAG" "$OUT/pmc_traffic_${ARCH}_$TAG.json" "$ARCH"
