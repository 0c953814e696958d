S="python -u tools/solve_time.py --reps 5 --shapes 3x400x128,6x300x128,7x256x128,5x500x128 --knobs persist=1 persist=0 persist=1 persist=0"
bash tools/gpu_steps.sh r06au ab 600 "$S"
