cd $GRAFT_REPO_ROOT
for L in "" build/exp/lib_plain.so; do
  FI_LIB_OVERRIDE=$L timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); k=d['kernel_ms_per_step']; print('$L', d['ms_per_step'], {x:k[x] for x in ['conv1_fwd','conv2_bwd','conv3_bwd']})"
done
export TMPDIR=/tmp; cd /tmp
FI_LIB_OVERRIDE=$GRAFT_REPO_ROOT/build/exp/lib_plain.so timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc_w_plain -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --profile-steps 1 --no-cpu-baseline > /dev/null 2>&1 || exit 2
python3 - <<'PY'
import csv,glob,collections
d=collections.defaultdict(list)
for f in glob.glob('/root/repo/gpurun_out/pmc_w_plain/**/*counter_collection.csv',recursive=True):
    for r in csv.DictReader(open(f)):
        for s in ['conv1_fwd_fr','conv2_bwd_fr','conv3_bwd_fr']:
            if s in r['Kernel_Name']: d[s].append(float(r['Counter_Value']))
print({k:sum(v)/len(v) for k,v in d.items()})
PY
