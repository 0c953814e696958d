#!/bin/bash
# Persistent-solve variant check (granule GroupNorm, opt 585 vs the default 73): correctness, tests, A/B, timeline.
mkdir -p gpurun_out/r03q
timeout -k 10 200 python tools/persist_check.py --nfe 32 73 585 > gpurun_out/r03q/check.log 2>&1 && tail -2 gpurun_out/r03q/check.log || exit 1
timeout -k 10 300 python -u -m pytest tests/test_persist_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03q/pytest.log 2>&1; tail -2 gpurun_out/r03q/pytest.log
bash tools/persist_ab.sh r03q 73 585 73 585 && bash tools/gpu_timeline.sh r03q 585
