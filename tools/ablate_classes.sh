#!/bin/bash
# In-graph cost of each denoiser kernel class: solve time with the class launched twice per step
# minus the baseline, divided by its launches per step.  Usage: tools/ablate_classes.sh TAG [bench args]
set -euo pipefail
TAG=$1; shift
mkdir -p gpurun_out/$TAG
for c in -1 0 1 2 3 4 5 6 7 8; do
  timeout -k 10 240 python bench.py --no-cpu-baseline --no-secondary --kernel-iters 1 --dup-class $c "$@" > gpurun_out/$TAG/d$c.json 2> gpurun_out/$TAG/d$c.err
done
python - gpurun_out/$TAG "$@" <<'PY'
import json, sys
d = sys.argv[1]
get = lambda c: json.loads(open(f"{d}/d{c}.json").read().strip().splitlines()[-1])
base = get(-1)
nfe = base["config"].get("nfe", 128)
names = [k["name"] for k in base["kernels"]]
per = [k["per_step"] for k in base["kernels"]]
print(f"baseline {base['ms_per_step']:.3f} ms/solve = {base['ms_per_step'] / nfe * 1e3:.1f} us/step")
tot = 0.0
for c in range(9):
    r = get(c)
    dus = (r["ms_per_step"] - base["ms_per_step"]) / nfe * 1e3
    tot += dus
    print(f"  class {c} {names[c]:28s} x{per[c]}/step: +{dus:7.1f} us/step -> {dus / per[c]:6.2f} us per launch")
print(f"  sum of class costs {tot:.1f} us/step")
PY
