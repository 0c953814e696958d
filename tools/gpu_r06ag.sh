A6="FLAMED_HIP_LIB=flamed-tts_amd/flamed/_native/libflamed_hip_d26.so"
A8="FLAMED_HIP_LIB=flamed-tts_amd/flamed/_native/libflamed_hip_d28.so"
S="python -u tools/solve_time.py --reps 10 --shapes 2x400x128,1x800x128,2x600x128"
bash tools/gpu_steps.sh r06ag \
 d10a 200 "$S" d6a 200 "$A6 $S" d8a 200 "$A8 $S" d10b 200 "$S" d6b 200 "$A6 $S" d8b 200 "$A8 $S" \
 tl400 200 "python -u tools/persist_timeline.py --frames 400 --out gpurun_out/r06ag/timeline_T400.txt" \
 tl800 200 "python -u tools/persist_timeline.py --frames 800 --out gpurun_out/r06ag/timeline_T800.txt"
