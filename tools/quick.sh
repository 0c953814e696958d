#!/bin/bash
# GPU quick check: full -m gpu suite, then bench at B=1 and B=64 with per-class kernel times.
# Usage: tools/quick.sh TAG [--no-tests]
set -euo pipefail
TAG=$1; shift
mkdir -p gpurun_out/$TAG
if [ "${1:-}" != "--no-tests" ]; then
  timeout -k 10 400 python -m pytest tests -m gpu -q -x > gpurun_out/$TAG/tests.log 2>&1 || { tail -30 gpurun_out/$TAG/tests.log; exit 1; }
  tail -1 gpurun_out/$TAG/tests.log
fi
summ() {
  python - "$1" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = " ".join(f"{k['name'][:10]}={k['us']}" for k in d["kernels"])
print(f"B={d['config']['batch_per_gpu']} ms/solve={d['ms_per_step']:.2f} frames/s={d['value']:.0f} | {ks}")
if d.get("secondary"):
    print("  secondary:", json.dumps(d["secondary"]))
PY
}
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/$TAG/b1.json 2> gpurun_out/$TAG/b1.err
summ gpurun_out/$TAG/b1.json
timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --batch 64 --steps 3 --warmup 1 > gpurun_out/$TAG/b64.json 2> gpurun_out/$TAG/b64.err
summ gpurun_out/$TAG/b64.json
