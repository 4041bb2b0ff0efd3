# round-5 GPU batch (A/B experiments): conv21 priority schedules (pr1: DMA waves at prio 1 while issuing; pr2: conv1-wgrad waves at prio 2 in phase 2)
AB_KERNELS=conv21_bwd,conv12_fwd ROUNDS=3 timeout -k 10 600 bash scripts/ab_rounds.sh prod build/ab/lib_pr1.so build/ab/lib_pr2.so > gpurun_out/ab_prio21.txt 2>&1
