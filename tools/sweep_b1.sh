#!/bin/bash
# B=1 knob sweep on the current tree: ms per 128-step solve for each flamed_tune variant.
mkdir -p gpurun_out/sweep
for v in "" "--bn32 0" "--small-stages 5" "--fuse-euler 0" ""; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-secondary --no-peaks --steps 8 $v > gpurun_out/sweep/o.json 2>/dev/null || { echo "fail: $v"; exit 1; }
  python -c "import json,sys;d=json.load(open('gpurun_out/sweep/o.json'));print('%-20s %.3f ms  step %.1f us' % (sys.argv[1] or 'default', d['ms_per_step'], d['step_us_graph']))" "$v"
done
