AB="FLAMED_HIP_LIB=flamed-tts_amd/flamed/_native/libflamed_hip_ab.so"
bash tools/gpu_steps.sh r06s \
 cur1 120 "python -u tools/solve_time.py --reps 20 --shapes 1x400x128,2x400x128" \
 ab1 120 "$AB python -u tools/solve_time.py --reps 20 --shapes 1x400x128,2x400x128" \
 cur2 120 "python -u tools/solve_time.py --reps 20 --shapes 1x400x128,2x400x128" \
 ab2 120 "$AB python -u tools/solve_time.py --reps 20 --shapes 1x400x128,2x400x128" \
 cur3 120 "python -u tools/solve_time.py --reps 20 --shapes 1x400x128,2x400x128" \
 ab3 120 "$AB python -u tools/solve_time.py --reps 20 --shapes 1x400x128,2x400x128"
