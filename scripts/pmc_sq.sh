#!/bin/bash
# pmc_sq.sh -- SQ stall counters of the frame-resident kernels, two passes of four SQ counters
# (counters only, no trace domains; each pass under its own hard time limit). Diagnostic only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
export TMPDIR=/tmp
cd /tmp
i=0
for SET in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
  i=$((i + 1))
  rm -rf "$OUT/pmcsq_$i"
  timeout -s KILL 120 rocprofv3 --pmc $SET --output-format csv -d "$OUT/pmcsq_$i" -o run \
      -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --profile-steps 1 --no-cpu-baseline \
      > "$OUT/pmcsq_$i.log" 2>&1
  rc=$?
  [ $rc -ne 0 ] && { echo "pmc pass $i rc=$rc"; tail -5 "$OUT/pmcsq_$i.log"; exit $rc; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
d = collections.defaultdict(lambda: collections.defaultdict(list))
for i in (1, 2):
    for f in glob.glob(f'{sys.argv[1]}/pmcsq_{i}/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            n = r['Kernel_Name']
            for s in ['conv12_fwd_fr', 'conv21_bwd_fr', 'conv3_bwd_fr', 'conv_fwd_fr<3>', 'vtrace_lds_kernel']:
                if s in n: d[s][r['Counter_Name']].append(float(r['Counter_Value']))
for k, cs in d.items():
    print(k, {c: f'{sum(v)/len(v):.4g}' for c, v in sorted(cs.items())})
PY
