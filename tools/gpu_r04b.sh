#!/bin/bash
# GPU box: persistent solve inside a captured graph, replayed (tools/capture_probe.py) under launch variants.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r04b
mkdir -p $OUT
step() { "$@"; rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "step rc=$rc: stopping"; exit $rc; fi; return 0; }
for args in "$@"; do
  echo "== $args"
  step timeout -k 10 120 python tools/capture_probe.py $args > $OUT/cap.log 2>&1
  cat $OUT/cap.log | grep -v "amdgpu.ids"
done
