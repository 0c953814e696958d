#!/bin/bash
# B=64 A/B: g8p_rows (0 = 128x128 ring) x x16
mkdir -p gpurun_out/r02h
timeout -k 10 400 python -u -m pytest tests/test_configs_gpu.py -k "cfg2" -v -s --timeout 200 --timeout-method thread > gpurun_out/r02h/tests.log 2>&1
rc=$?
grep -E "rel-L2|passed|failed|FAIL" gpurun_out/r02h/tests.log | tail -14
[ $rc -eq 0 ] || exit $rc
for g in 0 16384; do for x in 0 1; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --no-peaks --batch 64 --steps 3 --warmup 1 --x16 $x --g8p-rows $g > gpurun_out/r02h/b64_g${g}_x$x.json 2>/dev/null || exit 1
  python - gpurun_out/r02h/b64_g${g}_x$x.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1].split('/')[-1], "ms/solve", d["ms_per_step"], "step_us", d["step_us_graph"], " ".join(f"{k['name'][:10]}={k['us']}" for k in d["kernels"]))
PY
done; done
