AK="FLAMED_HIP_LIB=flamed-tts_amd/flamed/_native/libflamed_hip_abK.so"
S="python -u tools/solve_time.py --reps 3 --shapes 2x400x128,1x1500x128,4x400x128,1x2400x256,1x400x128"
bash tools/gpu_steps.sh r06ae \
 cur_a 200 "$S" ko_a 200 "$AK $S" cur_b 200 "$S" ko_b 200 "$AK $S"
