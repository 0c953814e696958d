bash tools/gpu_steps.sh r06e \
 timeline 300 "python -u tools/persist_timeline.py --frames 400 --nfe 16 --step 5 --out gpurun_out/r06e/timeline_T400.txt" \
 pmc_b1 900 "bash tools/pmc_mfma.sh r06e_b1" \
 pmc_b64 900 "bash tools/pmc_mfma.sh r06e_b64 --batch 64" \
 pmc_fp8 900 "bash tools/pmc_mfma.sh r06e_fp8 --config 4 --nfe 8"
