bash tools/gpu_steps.sh r06ap \
 t 300 "python -u -m pytest -x -v --timeout 180 --timeout-method thread -m gpu tests/test_persist_gpu.py -k 'seal'" \
 ab 600 "python -u tools/solve_time.py --reps 10 --shapes 1x400x128,2x400x128,1x2400x256 --knobs persist_opt=885322 persist_opt=1933898 persist_opt=885322 persist_opt=1933898"
