#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for i in 1 2; do
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/b$i.json || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/b$i.json')); k=d['kernel_ms_per_step']; print(d['ms_per_step'], {x: k[x] for x in list(k)[:7]})"
done
