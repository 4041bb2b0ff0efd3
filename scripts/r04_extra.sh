#!/bin/bash
# r04_extra.sh -- round-4 GPU step after round_check.sh: the FarmerLstm bench at the reference
# defaults and at B=512 T=100, a rocprofv3 kernel trace of the B=32 T=10 bench (dispatches per
# step), and the Atari bench line with one whole B=4096 CPU step as cpu_baseline (--cpu-full).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
timeout -k 10 300 python scripts/farmer_bench.py --configs 32x10,512x100 > "$OUT/farmer_r04.json" 2> "$OUT/farmer_r04.err"
rc=$?; echo "farmer rc=$rc"; cat "$OUT/farmer_r04.json"; [ $rc -ne 0 ] && { tail -5 "$OUT/farmer_r04.err"; exit $rc; }
export TMPDIR=/tmp
cd /tmp
rm -rf "$OUT/prof_farmer_r04"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_farmer_r04" -o run \
    -- python3 "$ROOT/scripts/farmer_bench.py" --configs 32x10 --no-cpu > "$OUT/prof_farmer_r04.log" 2>&1
rc=$?; echo "rocprof farmer rc=$rc"; [ $rc -ne 0 ] && exit $rc
cd "$ROOT"
# the CPU step is silent for ~1-2 min: a heartbeat file under gpurun_out shows it is alive
( while sleep 45; do date +%T >> "$OUT/heartbeat_r04.txt"; done ) &
HB=$!
timeout -k 10 900 python bench.py --arch atari --cpu-full > "$OUT/bench_atari_cpufull_r04.json" 2> "$OUT/bench_atari_cpufull_r04.err"
rc=$?; kill $HB; echo "bench cpu-full rc=$rc"; cat "$OUT/bench_atari_cpufull_r04.json"; [ $rc -ne 0 ] && { tail -5 "$OUT/bench_atari_cpufull_r04.err"; exit $rc; }
exit 0
