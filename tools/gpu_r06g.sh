bash tools/gpu_steps.sh r06g \
 tests 900 "python -u -m pytest tests/test_configs_gpu.py tests/test_denoiser_gpu.py -q --timeout 300 --timeout-method thread -m gpu" \
 ab_b64 300 "python -u tools/solve_time.py --reps 4 --shapes 64x400x128,32x400x128,4x400x128"
