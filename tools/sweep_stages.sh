#!/bin/bash
# bench ms/solve and per-class in-context us for each small-M pipeline depth.  Usage: tools/sweep_stages.sh TAG [bench args]
set -euo pipefail
TAG=$1; shift
mkdir -p gpurun_out/$TAG
for v in 3 5 7; do
  timeout -k 10 240 python bench.py --no-cpu-baseline --no-secondary --small-stages $v "$@" > gpurun_out/$TAG/s$v.json 2> gpurun_out/$TAG/s$v.err
  python - gpurun_out/$TAG/s$v.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = " ".join(f"{k['name'][:10]}={k['us']}" for k in d["kernels"])
print(f"stages={sys.argv[2]} ms/solve={d['ms_per_step']:.2f}  {ks}")
PY
done
