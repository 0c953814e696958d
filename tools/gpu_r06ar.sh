AP="FLAMED_HIP_LIB=flamed-tts_amd/flamed/_native/libflamed_hip_prev.so"
S="python -u tools/solve_time.py --reps 15 --shapes 1x400x128,2x400x128,1x2400x256"
bash tools/gpu_steps.sh r06ar cur_a 200 "$S" prev_a 200 "$AP $S" cur_b 200 "$S" prev_b 200 "$AP $S"
