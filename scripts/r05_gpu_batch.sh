# round-5 GPU batch (A/B experiments): heads weight gradient with packed FMAs (lib_hw) against the product
AB_KERNELS=heads_wgrad,heads_dgrad,heads_fwd,conv12_fwd ROUNDS=3 timeout -k 10 600 bash scripts/ab_rounds.sh prod build/ab/lib_hw.so > gpurun_out/ab_hw.txt 2>&1
