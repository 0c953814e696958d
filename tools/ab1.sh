#!/bin/bash
# B=1 A/B (dwgn_small) + denoiser GPU tests; usage: bash tools/ab1.sh TAG
TAG=${1:-r02k}
mkdir -p gpurun_out/$TAG
timeout -k 10 500 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_denoiser_gpu.py tests/test_configs_gpu.py > gpurun_out/$TAG/pytest.log 2>&1 || { tail -40 gpurun_out/$TAG/pytest.log; exit 1; }
tail -3 gpurun_out/$TAG/pytest.log
for v in "--dwgn-small 1" "--dwgn-small 0" "--dwgn-small 1"; do
  tag=$(echo $v | tr -d ' -')
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --no-peaks --steps 5 --warmup 2 $v > gpurun_out/$TAG/b1_$tag.json 2>/dev/null || exit 1
  python - gpurun_out/$TAG/b1_$tag.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1].split('/')[-1], "ms/solve", d["ms_per_step"], "step_us", d["step_us_graph"], " ".join(f"{k['name'][:10]}={k['us']}" for k in d["kernels"]))
PY
done
