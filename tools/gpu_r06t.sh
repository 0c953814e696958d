bash tools/gpu_steps.sh r06t \
 knobs 500 "python -u tools/solve_time.py --reps 12 --shapes 1x400x128 --knobs persist_opt=361034 persist_opt=362058 persist_opt=365130 persist_opt=361035 persist_opt=361034 persist_opt=362058 persist_opt=365130 persist_opt=361035"
