A8="FLAMED_HIP_LIB=flamed-tts_amd/flamed/_native/libflamed_hip_op8.so"
S="python -u tools/solve_time.py --reps 10 --shapes 1x400x128,2x400x128,1x2400x256"
bash tools/gpu_steps.sh r06aj \
 t 400 "python -u -m pytest -x -q --timeout 180 --timeout-method thread -m gpu tests/test_persist_gpu.py" \
 new_a 200 "$S" op8_a 200 "$A8 $S" new_b 200 "$S" op8_b 200 "$A8 $S"
