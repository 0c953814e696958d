bash tools/gpu_steps.sh r06aw \
 t 400 "python -u -m pytest -x -q --timeout 180 --timeout-method thread -m gpu tests/test_persist_gpu.py tests/test_configs_gpu.py" \
 ab 400 "python -u tools/solve_time.py --reps 3 --shapes 5x200x128,5x256x128 --knobs persist=1 persist=0"
