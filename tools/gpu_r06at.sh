S="python -u tools/solve_time.py --reps 3 --shapes 64x400x128,16x2400x256 --knobs split_batch=2 split_batch=3 split_batch=4 split_batch=3,g8p_rows=8192 split_batch=4,g8p_rows=6400 split_batch=2"
bash tools/gpu_steps.sh r06at ab 900 "$S"
