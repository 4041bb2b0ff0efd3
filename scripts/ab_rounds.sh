#!/bin/bash
# ab_rounds.sh LIB... -- interleaved A/B of experiment libraries (scripts/build_exp.sh) against the
# product library ("prod"): ROUNDS rounds (default 2) of one short Atari bench per library,
# printing ms/step and the top kernels (scripts/ab_libs.sh). The first failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 "${ROUNDS:-2}"); do
  echo "round $r"
  bash scripts/ab_libs.sh "$@" || exit 1
done
exit 0
