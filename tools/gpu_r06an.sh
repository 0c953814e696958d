A7="FLAMED_HIP_LIB=flamed-tts_amd/flamed/_native/libflamed_hip_d37.so"
A10="FLAMED_HIP_LIB=flamed-tts_amd/flamed/_native/libflamed_hip_d310.so"
S="python -u tools/solve_time.py --reps 8 --shapes 1x1500x128,4x300x128,2x600x128"
bash tools/gpu_steps.sh r06an \
 d8a 200 "$S" d7a 200 "$A7 $S" d10a 200 "$A10 $S" d8b 200 "$S" d7b 200 "$A7 $S" d10b 200 "$A10 $S"
