bash tools/gpu_steps.sh r06i \
 persist 600 "python -u -m pytest tests/test_persist_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu" \
 timing 400 "python -u tools/solve_time.py --reps 15 --shapes 1x400x128,2x400x128 && python -u tools/solve_time.py --reps 3 --shapes 1x2400x256" \
 multi 400 "python -u tools/solve_time.py --reps 5 --shapes 4x400x128,3x400x128,4x300x128,8x320x128,2x1000x128 --knobs persist_multi_ntw=5 persist_multi_ntw=2" \
 timeline 300 "python -u tools/persist_timeline.py --frames 400 --nfe 16 --step 5 --out gpurun_out/r06i/timeline_T400.txt"
