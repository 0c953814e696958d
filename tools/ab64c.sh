#!/bin/bash
# dwgn (whole-utterance depthwise conv + GroupNorm) parity + B=64 A/B (x dwgn x x16) + rocprof kernel trace
mkdir -p gpurun_out/r02j
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_denoiser_gpu.py -k "tuning_paths" > gpurun_out/r02j/pytest.log 2>&1 || { tail -30 gpurun_out/r02j/pytest.log; exit 1; }
tail -3 gpurun_out/r02j/pytest.log
for v in "--dwgn 0 --x16 0" "--dwgn 1 --x16 0" "--dwgn 0 --x16 1" "--dwgn 1 --x16 1" "--dwgn 1 --x16 0 --lnfold 0"; do
  tag=$(echo $v | tr -d ' -')
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --no-peaks --batch 64 --steps 3 --warmup 1 $v > gpurun_out/r02j/b64_$tag.json 2>/dev/null || exit 1
  python - gpurun_out/r02j/b64_$tag.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1].split('/')[-1], "ms/solve", d["ms_per_step"], "step_us", d["step_us_graph"], " ".join(f"{k['name'][:10]}={k['us']}" for k in d["kernels"]))
PY
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r02j/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-secondary --no-peaks --batch 64 --steps 1 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/r02j/prof.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/r02j/prof.log; exit 1; }
echo prof ok
