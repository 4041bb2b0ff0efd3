#!/bin/bash
# pmc_instmix.sh -- instruction mix, LDS and wait counters of the frame-resident conv kernels
# (conv21_bwd_fr, conv3_bwd_fr, conv12_fwd_fr, conv_fwd_fr<3>): one rocprofv3 --pmc pass per
# counter set (<= 8 SQ counters each, counters only, no trace domains), each under its own hard
# time limit, over a short bench run. Summary: gpurun_out/pmc_instmix_$TAG.json
# (scripts/pmc_instmix.py). A pass rejected by rocprofv3 (unknown counter: rc 1) is skipped; a
# timeout / abort / fault ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
TAG=${TAG:-r02}
export FI_BENCH_ARCH=${ARCH:-atari}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/rocprof_avail_$TAG.txt" 2>&1 || true
i=0
for SET in "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_BUSY_CYCLES" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_CVT SQ_ACTIVE_INST_FLAT SQ_ACTIVE_INST_SCA" \
           "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY"; do
  i=$((i + 1))
  rm -rf "$OUT/pmcmix_$i"
  timeout -s KILL 90 rocprofv3 --pmc $SET --output-format csv -d "$OUT/pmcmix_$i" -o run \
      -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --profile-steps 1 --sustain-seconds 0 --no-cpu-baseline \
      > "$OUT/pmcmix_$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc: $SET"
  if [ $rc -ge 124 ]; then tail -5 "$OUT/pmcmix_$i.log"; exit $rc; fi
done
python3 "$ROOT/scripts/pmc_instmix.py" "$OUT" "$OUT/pmc_instmix_$TAG.json"
