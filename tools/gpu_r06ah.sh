A7="FLAMED_HIP_LIB=flamed-tts_amd/flamed/_native/libflamed_hip_d27.so"
A9="FLAMED_HIP_LIB=flamed-tts_amd/flamed/_native/libflamed_hip_d29.so"
S="python -u tools/solve_time.py --reps 10 --shapes 2x400x128,1x800x128,2x1000x128"
bash tools/gpu_steps.sh r06ah \
 d8a 200 "$S" d7a 200 "$A7 $S" d9a 200 "$A9 $S" d8b 200 "$S" d7b 200 "$A7 $S" d9b 200 "$A9 $S"
