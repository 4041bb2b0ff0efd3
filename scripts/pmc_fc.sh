#!/bin/bash
# pmc_fc.sh -- rocprofv3 counter passes over build/fc_bench for the variants matching $1
# (one --pmc pass per counter set, each under its own hard limit). Output: gpurun_out/pmcfc_*
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for SET in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_VMEM" \
           "GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_LDS" \
           "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i + 1))
  rm -rf "$OUT/pmcfc_$i"
  timeout -s KILL 90 rocprofv3 --pmc $SET --output-format csv -d "$OUT/pmcfc_$i" -o run \
      -- "$ROOT/build/fc_bench" 1 413696 "$1" > "$OUT/pmcfc_$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc: $SET"
  if [ $rc -ge 124 ]; then tail -5 "$OUT/pmcfc_$i.log"; exit $rc; fi
done
exit 0
