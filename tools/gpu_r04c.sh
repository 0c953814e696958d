#!/bin/bash
# GPU box: persistent-solve tests, then the default bench line (B = 1) and a stamped timeline.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04c}
mkdir -p $OUT
step() { "$@"; rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "step rc=$rc: stopping"; exit $rc; fi; return 0; }
step timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_persist_gpu.py > $OUT/persist.log 2>&1
tail -4 $OUT/persist.log
step timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
python -c "import json; d=json.load(open('$OUT/bench.json')); print('value', d['value'], 'ms', d['ms_per_step'], 'roof', d['roofline']['frac'], d['roofline']['launch_us'])"
step timeout -k 10 120 python tools/persist_timeline.py --out $OUT/timeline.txt > $OUT/tl.log 2>&1
head -2 $OUT/timeline.txt
