bash tools/gpu_steps.sh r06f \
 ab_b64 300 "python -u tools/solve_time.py --reps 4 --shapes 64x400x128,32x400x128,4x400x128" \
 tests 900 "python -u -m pytest tests/test_configs_gpu.py tests/test_denoiser_gpu.py -x -q --timeout 300 --timeout-method thread -m gpu" \
 pmc_b64 900 "bash tools/pmc_mfma.sh r06f_b64 --batch 64"
