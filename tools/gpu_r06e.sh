bash tools/gpu_steps.sh r06e \
 configs 900 "python -u -m pytest tests/test_configs_gpu.py -x -v --timeout 300 --timeout-method thread -m gpu -k 'concurrent or split_batch'" \
 pmc_b1 900 "bash tools/pmc_mfma.sh r06e_b1" \
 pmc_b64 900 "bash tools/pmc_mfma.sh r06e_b64 --batch 64" \
 pmc_fp8 900 "bash tools/pmc_mfma.sh r06e_fp8 --config 4"
