#!/bin/bash
# PVA direct-buffer path: PVA / end-to-end / ops GPU tests, then the secondary bench rows.
mkdir -p gpurun_out/r03y
timeout -k 10 300 python -u -m pytest tests/test_pva_gpu.py tests/test_flamed_gpu.py tests/test_ops_gpu.py tests/test_synthesize_gpu.py -x -q --timeout 180 --timeout-method thread > gpurun_out/r03y/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r03y/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-peaks > gpurun_out/r03y/bench.json 2> gpurun_out/r03y/bench.err || exit 1
python -c "
import json; s=json.load(open('gpurun_out/r03y/bench.json'))['secondary']
[print(k, {kk: v for kk, v in s[k].items() if kk not in ('note', 'duration_flips')}) for k in ('pva_flow_lr', 'prior_transformer', 'end_to_end', 'end_to_end_5s')]"
