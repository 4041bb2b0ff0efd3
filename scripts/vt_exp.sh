#!/bin/bash
# V-trace kernel A/B session: parity tests on the product library, then timing of the
# experiment builds in build/exp (scripts/build_vt.sh) and the streaming calibration probe.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 200 python -m pytest -q -x tests/test_gpu_vtrace.py --timeout 120 > gpurun_out/vt_pytest.txt 2>&1 || { tail -30 gpurun_out/vt_pytest.txt; exit 1; }
tail -2 gpurun_out/vt_pytest.txt
[ -x build/exp/stream_probe ] && { timeout -k 10 60 build/exp/stream_probe > gpurun_out/stream.txt 2>&1 || exit 1; }
libs=""
for l in ${VT_LIBS:-base pf base pf}; do libs="$libs --lib build/exp/libvt_$l.so"; done
timeout -k 10 120 python scripts/vtrace_bench.py $libs > gpurun_out/vt.txt 2>&1 || exit 1
for l in ${VT_STAMPS:-}; do
  timeout -k 10 120 python scripts/vtrace_bench.py --lib build/exp/libvt_$l.so --stamps >> gpurun_out/vt_st.txt 2>&1 || exit 1
done
cat gpurun_out/vt.txt gpurun_out/vt_st.txt 2>/dev/null
