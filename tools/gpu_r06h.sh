bash tools/gpu_steps.sh r06h \
 persist 600 "python -u -m pytest tests/test_persist_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu" \
 timing 400 "python -u tools/solve_time.py --reps 15 --shapes 1x400x128,2x400x128 && python -u tools/solve_time.py --reps 3 --shapes 1x2400x256,64x400x128" \
 tests 900 "python -u -m pytest tests/test_configs_gpu.py tests/test_denoiser_gpu.py -q --timeout 300 --timeout-method thread -m gpu" \
 timeline 300 "python -u tools/persist_timeline.py --frames 400 --nfe 16 --step 5 --out gpurun_out/r06h/timeline_T400.txt"
