bash tools/gpu_steps.sh r06n \
 sweep 600 "python -u tools/solve_time.py --reps 3 --shapes 64x400x128 --knobs '' x16=1 split_batch=1 split_batch=4 g8p_rows=6400 split_batch=4,g8p_rows=6400 ''" \
 sweep16 300 "python -u tools/solve_time.py --reps 2 --shapes 16x2400x256 --knobs '' split_batch=1 g8p_rows=19200"
