#!/bin/bash
# Split-K sweep for the small-M denoiser GEMMs: bench ms/solve and per-kernel in-context times.
# Usage: tools/sweep_split.sh TAG "target:max ..." [bench args]
set -euo pipefail
TAG=$1; shift
VARIANTS=$1; shift
mkdir -p gpurun_out/$TAG
for v in $VARIANTS; do
  t=${v%%:*}; m=${v##*:}
  timeout -k 10 240 python bench.py --no-cpu-baseline --no-secondary --splitk-target $t --splitk-max $m "$@" > gpurun_out/$TAG/b_${t}_${m}.json 2> gpurun_out/$TAG/b_${t}_${m}.err
  python - gpurun_out/$TAG/b_${t}_${m}.json "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = " ".join(f"{k['name'][:10]}={k['us']}" for k in d["kernels"])
print(f"{sys.argv[2]:>10s} ms/solve={d['ms_per_step']:.2f}  {ks}")
PY
done
