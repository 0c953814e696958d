bash tools/gpu_steps.sh r06v \
 t800 300 "python -u tools/persist_timeline.py --frames 800 --nfe 16 --step 5 --out gpurun_out/r06v/timeline_T800.txt" \
 t2400 300 "python -u tools/persist_timeline.py --frames 2400 --nfe 16 --step 5 --out gpurun_out/r06v/timeline_T2400.txt"
