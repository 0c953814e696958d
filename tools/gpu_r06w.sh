bash tools/gpu_steps.sh r06w \
 ab 600 "python -u tools/solve_time.py --reps 5 --shapes 1x2400x256,2x400x128,4x400x128,1x800x128 --knobs persist_opt=361034 persist_opt=98890 persist_opt=361034 persist_opt=98890"
