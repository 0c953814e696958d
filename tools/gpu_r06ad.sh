AC="FLAMED_HIP_LIB=flamed-tts_amd/flamed/_native/libflamed_hip_abC.so"
S="python -u tools/solve_time.py --reps 3 --shapes 1x3000x256,4x800x128,4x1024x128,8x500x128"
bash tools/gpu_steps.sh r06ad \
 d2a 200 "$S" d3a 200 "$AC $S" d2b 200 "$S" d3b 200 "$AC $S"
