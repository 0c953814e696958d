bash tools/gpu_steps.sh r06u \
 ab 500 "python -u tools/solve_time.py --reps 15 --shapes 1x400x128,2x400x128 --knobs persist_opt=361034 persist_opt=885322 persist_opt=361034 persist_opt=885322 persist_opt=361034 persist_opt=885322"
