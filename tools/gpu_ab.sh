#!/bin/bash
# GPU box: B = 1 persistent-solve A/B over persist_opt values (bench.py, 10 timed solves each, no secondary
# rows) plus one stamped timeline per value.  Usage: bash tools/gpu_ab.sh TAG OPT [OPT ...]
set -u
TAG=${1:-ab}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for o in "$@"; do
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-peaks --persist-opt $o > $OUT/bench_o$o.json 2> $OUT/bench_o$o.err || { tail -20 $OUT/bench_o$o.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/bench_o$o.json')); print('opt', $o, 'ms/solve', d['ms_per_step'], 'persistent runs', d['persistent']['runs'], 'kernel ms', d['roofline'].get('launch_us'))"
  timeout -k 10 120 python tools/persist_timeline.py --opt $o --out $OUT/timeline_o$o.txt > $OUT/tl_o$o.log 2>&1 || { tail -20 $OUT/tl_o$o.log; exit 1; }
  head -2 $OUT/timeline_o$o.txt
done
