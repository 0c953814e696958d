#!/bin/bash
# GPU box: persistent-solve timelines (stamps build) for the given persist_opt values.
# Usage: bash tools/gpu_timeline.sh TAG OPT [OPT ...]
set -u
TAG=${1:-tl}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for o in "$@"; do
  timeout -k 10 120 python tools/persist_timeline.py --opt $o --out $OUT/timeline_o$o.txt > $OUT/o$o.log 2>&1 || { tail -20 $OUT/o$o.log; exit 1; }
  head -3 $OUT/timeline_o$o.txt
done
