bash tools/gpu_steps.sh r06ac \
 t 400 "python -u -m pytest -x -v --timeout 180 --timeout-method thread -m gpu tests/test_persist_gpu.py -k 'multi_chunk'" \
 ab 700 "python -u tools/solve_time.py --reps 3 --shapes 1x3000x256,4x800x128,3x800x128,4x1024x128,8x500x128,1x2400x256 --knobs persist_ntw=8,persist_multi_ntw=8 persist=0 persist_ntw=8,persist_multi_ntw=8"
