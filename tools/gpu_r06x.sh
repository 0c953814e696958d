bash tools/gpu_steps.sh r06x \
 t 300 "python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_persist_gpu.py -k 'multi_chunk_variants or multi_counter or padded'" \
 ab 600 "python -u tools/solve_time.py --reps 5 --shapes 1x2400x256,2x400x128,4x400x128,1x800x128,8x300x64 --knobs persist_opt=361034 persist_opt=885322 persist_opt=361034 persist_opt=885322"
