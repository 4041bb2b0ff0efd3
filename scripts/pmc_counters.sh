#!/bin/bash
# pmc_counters.sh COUNTER... -- one rocprofv3 --pmc pass per counter over a short bench run
# (counters only, no trace domains), then the mean value per FR kernel. Diagnostic only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
export TMPDIR=/tmp
cd /tmp
for C in "$@"; do
  rm -rf "$OUT/pmcc_$C"
  timeout -k 10 600 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmcc_$C" -o run \
      -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --profile-steps 1 --no-cpu-baseline \
      > "$OUT/pmcc_$C.log" 2>&1
  rc=$?
  [ $rc -ne 0 ] && { echo "pmc $C rc=$rc"; exit $rc; }
  python3 - "$OUT/pmcc_$C" "$C" <<'PY'
import csv, glob, sys, collections
d = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if r['Counter_Name'] != sys.argv[2]: continue
        n = r['Kernel_Name']
        for s in ['conv1_fwd_fr', 'conv1_wgrad_fr', 'conv2_bwd_fr', 'conv3_bwd_fr', 'conv_fwd_fr<2>', 'conv_fwd_fr<3>']:
            if s in n: d[s].append(float(r['Counter_Value']))
print(sys.argv[2], {k: f'{sum(v)/len(v):.4g}' for k, v in d.items()})
PY
done
