bash tools/gpu_steps.sh r06av \
 t 400 "python -u -m pytest -x -q --timeout 180 --timeout-method thread -m gpu tests/test_persist_gpu.py" \
 ab 500 "python -u tools/solve_time.py --reps 3 --shapes 5x500x128,5x300x128,3x800x128,6x300x128 --knobs persist=1 persist=0"
