#!/bin/bash
# pmc_round.sh -- every counter pass the bench line and DESIGN.md cite, for the CURRENT sources
# (each summary is stamped with freeimpala_amd/build_info.source_hash(); bench.py attaches only
# matching ones): HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes) and MFMA busy + clock
# for the Atari and MLP lines, the instruction-mix passes for the Atari conv kernels.
# Counters only (no trace domains); every pass under its own time limit; a failure ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r03}
for A in atari mlp; do
  ARCH=$A TAG=$TAG bash scripts/pmc_pass.sh || exit $?
  ARCH=$A TAG=$TAG bash scripts/pmc_mfma.sh || exit $?
done
if [ "${INSTMIX:-1}" = 1 ]; then
  ARCH=atari TAG=$TAG bash scripts/pmc_instmix.sh || exit $?
fi
ls -la gpurun_out/pmc_*_$TAG.json
