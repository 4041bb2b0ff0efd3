# round-5 GPU batch: full-length bench (20 steps after 5 warm-up) of the final tree and of lib_nt (non-temporal stores), interleaved, same box
for r in 1 2; do
  for L in "" build/ab/lib_nt.so; do
    FI_LIB_OVERRIDE=$L timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/full_ab.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/full_ab.json')); k=d['kernel_ms_per_step']; print('${L:-prod}', d['ms_per_step'], {x: k[x] for x in ('conv21_bwd','conv12_fwd','conv3_bwd','conv3_fwd')})" >> gpurun_out/full_ab.txt
  done
done
