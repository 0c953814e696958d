bash tools/gpu_steps.sh r06p \
 persist 600 "python -u -m pytest tests/test_persist_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu" \
 timing 300 "python -u tools/solve_time.py --reps 15 --shapes 1x400x128,2x400x128,4x100x128,8x64x128,4x400x128"
