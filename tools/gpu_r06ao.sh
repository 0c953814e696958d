bash tools/gpu_steps.sh r06ao \
 t 400 "python -u -m pytest -x -q --timeout 180 --timeout-method thread -m gpu tests/test_persist_gpu.py tests/test_configs_gpu.py" \
 ab 300 "python -u tools/solve_time.py --reps 5 --shapes 1x1500x128,4x300x128,2x600x128,1x400x128"
