AA="FLAMED_HIP_LIB=flamed-tts_amd/flamed/_native/libflamed_hip_abA.so"
AB="FLAMED_HIP_LIB=flamed-tts_amd/flamed/_native/libflamed_hip_abB.so"
S="python -u tools/solve_time.py --reps 5 --shapes 1x1500x128,4x300x128,4x400x128,2x1000x128,1x2400x256"
bash tools/gpu_steps.sh r06aa \
 cur_a 200 "$S" A_a 200 "$AA $S" B_a 200 "$AB $S" cur_b 200 "$S" A_b 200 "$AA $S" B_b 200 "$AB $S"
