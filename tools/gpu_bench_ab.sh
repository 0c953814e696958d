#!/bin/bash
# GPU box: quick B = 1 A/B of persist_opt values (bench.py, no secondary rows), after the persistent-solve tests.
# Usage: bash tools/gpu_bench_ab.sh TAG OPT [OPT ...]
set -u
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
step() { "$@"; rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "step rc=$rc: stopping"; exit $rc; fi; return 0; }
step timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_persist_gpu.py > $OUT/persist.log 2>&1
tail -2 $OUT/persist.log
for o in "$@"; do
  step timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-secondary --no-peaks --persist-opt $o > $OUT/bench_o$o.json 2> $OUT/bench_o$o.err
  python -c "import json; d=json.load(open('$OUT/bench_o$o.json')); print('opt', $o, 'ms/solve', d['ms_per_step'], 'kernel us', d['roofline'].get('launch_us'))"
done
