#!/bin/bash
# PVA batching + bf16 prior decoders: the affected GPU tests, then the secondary bench rows and timelines.
set -u
OUT=gpurun_out/${1:-r03n}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_pva_gpu.py tests/test_prior_gpu.py tests/test_flamed_gpu.py tests/test_facodec_enc_gpu.py -x -v -s --timeout 180 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; grep -E 'passed|failed|rel-L2|PASS|FAIL' $OUT/pytest.log | tail -40; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/pva_timeline.py --out $OUT/pva_tl60.txt && timeout -k 10 120 python tools/pva_timeline.py --phonemes 285 --out $OUT/pva_tl285.txt || exit 1
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-peaks > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python -c "
import json; p=json.load(open('$OUT/bench.json')); s=p['secondary']
print(p['ms_per_step']); [print(k, s.get(k)) for k in ('pva_flow_lr','prior_transformer','end_to_end','end_to_end_5s')]"
