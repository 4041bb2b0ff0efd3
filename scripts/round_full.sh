#!/bin/bash
# round_full.sh TAG -- the stamped counter passes for the current sources (scripts/pmc_round.sh),
# copied into profiles/ on the box so the bench lines of the same call attach them, then
# scripts/round_check.sh (every GPU test, smoke, Atari + MLP bench lines, kernel-trace stats).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r03}
TAG=$TAG bash scripts/pmc_round.sh > gpurun_out/pmc_round_$TAG.txt 2>&1
rc=$?; echo "pmc round rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/pmc_round_$TAG.txt; exit $rc; }
for f in pmc_traffic_atari pmc_traffic_mlp pmc_mfma_atari pmc_mfma_mlp; do
  cp gpurun_out/${f}_$TAG.json profiles/${TAG}_$f.json || exit 1
done
cp gpurun_out/pmc_instmix_$TAG.json profiles/${TAG}_pmc_instmix_atari.json || exit 1
bash scripts/round_check.sh $TAG
