# round-5 GPU batch (A/B experiments): the frame-resident kernels' output stores with the default cache policy (lib_plain)
FI_LIB_OVERRIDE=$PWD/build/ab/lib_plain.so ARCH=atari TAG=plain bash scripts/pmc_pass.sh > gpurun_out/pmc_plain.txt 2>&1 || exit 1
AB_KERNELS=conv12_fwd,conv3_fwd,conv3_bwd,conv21_bwd ROUNDS=3 timeout -k 10 600 bash scripts/ab_rounds.sh prod build/ab/lib_plain.so > gpurun_out/ab_plain.txt 2>&1
