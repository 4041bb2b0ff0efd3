# round-5 GPU batch (A/B experiments): fc weight gradient with the leftover slice's tiles dealt to XCDs in blocks (lib_wg)
FI_LIB_OVERRIDE=$PWD/build/ab/lib_wg.so ARCH=atari TAG=wg bash scripts/pmc_pass.sh > gpurun_out/pmc_wg.txt 2>&1 || exit 1
AB_KERNELS=fc_wgrad,fc_dgrad,fc_fwd ROUNDS=3 timeout -k 10 600 bash scripts/ab_rounds.sh prod build/ab/lib_wg.so > gpurun_out/ab_wg.txt 2>&1
