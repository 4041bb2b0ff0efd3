# round-5 GPU batch (A/B experiments): conv21 with the raw-frame conversion inside the conv2 weight-gradient MFMA loop (lib_cvms)
timeout -k 10 200 env FI_LIB_OVERRIDE=build/ab/lib_cvms.so python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_atari.py -k "conv21 or steady_state or frame_resident" > gpurun_out/cvms_tests.log 2>&1 || exit 1
AB_KERNELS=conv21_bwd,conv12_fwd ROUNDS=3 timeout -k 10 600 bash scripts/ab_rounds.sh prod build/ab/lib_cvms.so > gpurun_out/ab_cvms.txt 2>&1
