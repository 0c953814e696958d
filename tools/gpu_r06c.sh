bash tools/gpu_steps.sh r06c \
 persist 600 "python -u -m pytest tests/test_persist_gpu.py -v --timeout 200 --timeout-method thread -m gpu" \
 ab_rowpart 300 "python -u tools/solve_time.py --reps 15 --shapes 1x400x128,2x400x128 --knobs persist_opt=361032 persist_opt=361034 persist_opt=361032 persist_opt=361034" \
 ab_pad 300 "python -u tools/solve_time.py --reps 8 --shapes 3x400x128,4x400x128,6x100x128,8x100x128 --knobs persist_pad=1 persist_pad=0" \
 ab_pk_def 300 "python -u tools/solve_time.py --reps 15 --shapes 1x400x128 --knobs persist_opt=361032 && python -u tools/solve_time.py --reps 4 --shapes 64x400x128" \
 ab_pk_nopk 300 "FLAMED_HIP_LIB=flamed-tts_amd/flamed/_native/libflamed_hip_nopk.so python -u tools/solve_time.py --reps 15 --shapes 1x400x128 --knobs persist_opt=361032 && FLAMED_HIP_LIB=flamed-tts_amd/flamed/_native/libflamed_hip_nopk.so python -u tools/solve_time.py --reps 4 --shapes 64x400x128" \
 ab_pk_def2 300 "python -u tools/solve_time.py --reps 15 --shapes 1x400x128 --knobs persist_opt=361032 && python -u tools/solve_time.py --reps 4 --shapes 64x400x128"
