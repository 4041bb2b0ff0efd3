# round-5 GPU batch (A/B experiments): conv12 conversion split + priority, fc dgrad XCD-row tile order
timeout -k 10 200 env FI_LIB_OVERRIDE=build/ab/lib_dgx.so python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_atari.py -k "fc or steady_state" > gpurun_out/dgx_tests.log 2>&1 || exit 1
ROUNDS=2 timeout -k 10 600 bash scripts/ab_rounds.sh prod build/ab/lib_c12_1340.so build/ab/lib_c12_1340_p1.so build/ab/lib_c12_1340_p2.so build/ab/lib_c12_2340.so build/ab/lib_dgx.so > gpurun_out/ab_c12prio.txt 2>&1
