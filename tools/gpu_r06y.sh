AB="FLAMED_HIP_LIB=flamed-tts_amd/flamed/_native/libflamed_hip_ab.so"
S="python -u tools/solve_time.py --reps 5 --shapes 1x2400x256,2x400x128,4x400x128,1x800x128,8x300x64"
bash tools/gpu_steps.sh r06y \
 cur1 200 "$S" ab1 200 "$AB $S" cur2 200 "$S" ab2 200 "$AB $S"
