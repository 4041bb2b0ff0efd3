#!/bin/bash
# Config #5 shape on one box: N actor ranks (host cores, MPI shared memory) feeding the device
# learner on rank 0 (tools/fi_freeimpala_mpi.cpp). Prints rank 0's JSON line (mpi.e2e_env_steps_per_s,
# receive GB/s, learner metrics). The actors generate the 1 KiB records on the CPU (normal
# draws), which is what bounds this run, not the learner.
#   ACTORS=16 M=512 ITERS=64 ARCH=mlp scripts/mpi_e2e.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ACTORS=${ACTORS:-16}
M=${M:-512}
ITERS=${ITERS:-64}
T=${T:-100}
ARCH=${ARCH:-mlp}
OUT=${OUT:-gpurun_out/mpi_e2e_a${ACTORS}_m${M}.json}
mkdir -p "$(dirname "$OUT")"
export HYDRA_LAUNCHER=fork
timeout -k 10 ${E2E_TIMEOUT:-300} /opt/conda/bin/mpiexec -n $((ACTORS + 1)) build/fi_freeimpala_mpi \
    --players 1 --iterations "$ITERS" --buffer-capacity $((2 * M)) --batch-size "$M" \
    --seq-length "$T" --entry-size $((T + 1)) --game-steps $((T + 1)) --agent-time 0 \
    --checkpoint-freq 0 --checkpoint-location /tmp/fi_mpi_e2e_ck --learner-arch "$ARCH" --log-level warn \
    > "$OUT.log" 2>&1
rc=$?
tail -1 "$OUT.log" > "$OUT"
echo "mpi_e2e rc=$rc"; cat "$OUT"
exit $rc
