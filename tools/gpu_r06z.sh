A16="FLAMED_HIP_LIB=flamed-tts_amd/flamed/_native/libflamed_hip_ab16.so"
A12="FLAMED_HIP_LIB=flamed-tts_amd/flamed/_native/libflamed_hip_ab12.so"
S="python -u tools/solve_time.py --reps 5 --shapes 1x2400x256,4x400x128,8x300x64,2x1000x128"
bash tools/gpu_steps.sh r06z \
 r20a 200 "$S" r16a 200 "$A16 $S" r12a 200 "$A12 $S" r20b 200 "$S" r16b 200 "$A16 $S" r12b 200 "$A12 $S"
