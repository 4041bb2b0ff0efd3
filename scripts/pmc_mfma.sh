#!/bin/bash
# pmc_mfma.sh -- MFMA utilisation and effective clock of the step's kernels: one rocprofv3 pass
# with SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE (counters only, plus the kernel trace for
# durations), summarised by scripts/pmc_mfma.py into gpurun_out/pmc_mfma_$TAG.json.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
TAG=${TAG:-r01}
ARCH=${ARCH:-atari}
export FI_BENCH_ARCH=$ARCH
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
rm -rf "$OUT/pmc_mfma_${ARCH}_$TAG"
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv \
    -d "$OUT/pmc_mfma_${ARCH}_$TAG" -o run -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --profile-steps 1 --sustain-seconds 0 \
    --no-cpu-baseline > "$OUT/pmc_mfma_${ARCH}_$TAG.log" 2>&1
rc=$?
[ $rc -ne 0 ] && { echo "pmc rc=$rc"; tail -5 "$OUT/pmc_mfma_${ARCH}_$TAG.log"; exit $rc; }
python3 "$ROOT/scripts/pmc_mfma.py" "$OUT/pmc_mfma_${ARCH}_$TAG" "$OUT/pmc_mfma_${ARCH}_$TAG.json"
