# round-5 GPU batch (A/B experiments): conv12 conversion unit splits (NCA, NC, NA) against the product (1, 3, 4)
for L in 352 452 252; do timeout -k 10 200 env FI_LIB_OVERRIDE=build/ab/lib_u$L.so python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_atari.py -k "conv12 or steady_state" > gpurun_out/u_tests_$L.log 2>&1 || exit 1; done
ROUNDS=2 timeout -k 10 600 bash scripts/ab_rounds.sh prod build/ab/lib_u243.so build/ab/lib_u343.so build/ab/lib_u352.so build/ab/lib_u452.so build/ab/lib_u252.so > gpurun_out/ab_units2.txt 2>&1
