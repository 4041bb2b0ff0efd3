# round-5 GPU batch (A/B experiments): conv3 forward on 32x32x16 MFMAs with two accumulator chains (read-ahead 4 / 8)
AB_KERNELS=conv3_fwd,conv12_fwd ROUNDS=2 timeout -k 10 600 bash scripts/ab_rounds.sh prod build/ab/lib_wide2.so build/ab/lib_wide2p8.so > gpurun_out/ab_wide2.txt 2>&1
