# round-5 GPU batch (A/B experiments): conv3_bwd with the issuing waves' reshuffle + DMA after their MFMAs (lib_c3o1)
timeout -k 10 200 env FI_LIB_OVERRIDE=build/ab/lib_c3o1.so python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_atari.py -k "steady_state or frame_resident or fc_path" > gpurun_out/c3o_tests.log 2>&1
timeout -k 10 120 python scripts/grads_dump.py gpurun_out/g_prod.npy && FI_LIB_OVERRIDE=build/ab/lib_c3o1.so timeout -k 10 120 python scripts/grads_dump.py gpurun_out/g_c3o1.npy || exit 1
python -c "import numpy as np; a=np.load('gpurun_out/g_prod.npy'); b=np.load('gpurun_out/g_c3o1.npy'); print('bit-identical grads:', np.array_equal(a,b))" > gpurun_out/c3o_cmp.txt
AB_KERNELS=conv3_bwd,conv21_bwd,conv12_fwd ROUNDS=3 timeout -k 10 600 bash scripts/ab_rounds.sh prod build/ab/lib_c3o1.so > gpurun_out/ab_c3o.txt 2>&1
