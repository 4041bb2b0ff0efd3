# round-5 GPU batch (A/B experiments): conv3 forward with one 32x32x16 MFMA per 16-deep k-step (lib_wide)
timeout -k 10 400 env FI_LIB_OVERRIDE=build/ab/lib_wide.so python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_atari.py > gpurun_out/wide_tests.log 2>&1 || exit 1
AB_KERNELS=conv3_fwd,conv12_fwd,conv21_bwd ROUNDS=3 timeout -k 10 600 bash scripts/ab_rounds.sh prod build/ab/lib_wide.so > gpurun_out/ab_wide.txt 2>&1
