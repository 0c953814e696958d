#!/bin/bash
# GPU box: small metadata-mode batches (B = 2 / 4 / 8 equal-length utterances, nfe 128) with the persistent
# solve (persist_multi 1) vs the graph of launches (persist_multi 0).  Usage: bash tools/gpu_multi_ab.sh TAG
set -u
export TMPDIR=/tmp
TAG=${1:-multi}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for bt in "2 200" "4 100" "8 64" "2 400" "4 400"; do
  set -- $bt
  for pm in 0 1; do
    timeout -k 10 200 python bench.py --batch $1 --frames $2 --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --no-peaks --no-configs3 --persist-multi $pm > $OUT/m_${1}_${2}_$pm.json 2> $OUT/m_${1}_${2}_$pm.err
    rc=$?; if [ $rc -ne 0 ]; then echo "bench rc=$rc (B=$1 T=$2 pm=$pm)"; tail -5 $OUT/m_${1}_${2}_$pm.err; exit $rc; fi
    python -c "import json; d=json.load(open('$OUT/m_${1}_${2}_$pm.json')); print('B=$1 T=$2 persist_multi=$pm', 'ms/solve', d['ms_per_step'], 'kernel', d['roofline'].get('kernel'))"
  done
done
