#!/bin/bash
# GPU box: configs[2] (B = 64, T = 400, nfe = 128) A/B of knob sets (bench.py --config 2, no secondary rows),
# printing ms per solve and the per-class in-graph kernel times.  Usage: bash tools/gpu_b64_ab.sh TAG "ARGS" ["ARGS" ...]
set -u
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
i=0
for args in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --config 2 --steps 3 --warmup 1 --kernel-iters 5 --no-cpu-baseline --no-secondary --no-peaks $args > $OUT/b64_$i.json 2> $OUT/b64_$i.err
  rc=$?; if [ $rc -ne 0 ]; then echo "bench rc=$rc ($args)"; tail -5 $OUT/b64_$i.err; exit $rc; fi
  python -c "import json; d=json.load(open('$OUT/b64_$i.json')); print('[$args]', 'ms/solve', d['ms_per_step'], 'step_us', d['step_us_graph'], ' '.join(f\"{k['name']}={k['us']}\" for k in d['kernels']))"
done
