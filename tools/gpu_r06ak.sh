bash tools/pmc_mfma.sh r06ak_T2400 --frames 2400 --nfe 256 && bash tools/pmc_mfma.sh r06ak_B4T800 --batch 4 --frames 800 --nfe 128
