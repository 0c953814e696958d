S="python -u tools/solve_time.py --reps 5 --shapes 1x400x128,2x400x128,1x2400x256,4x800x128,4x400x128 --knobs persist_opt=885322 persist_opt=885314 persist_opt=885322 persist_opt=885314"
bash tools/gpu_steps.sh r06al ab 900 "$S"
