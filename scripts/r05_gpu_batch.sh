# round-5 GPU batch: fc dgrad tiles in column pairs per workgroup (OPT 256), stand-alone timing + PMC
timeout -k 10 300 ./build/fc_bench 5 413696 dgrd > gpurun_out/fcb_pairs.txt 2>&1 || exit 1
timeout -k 10 400 bash scripts/pmc_fc.sh dgrd > gpurun_out/pmcfc_pairs.txt 2>&1
