#!/bin/bash
# bf16 prior decoders with split-K: prior / end-to-end GPU tests, then decode timings.
mkdir -p gpurun_out/r03v
timeout -k 10 300 python -u -m pytest tests/test_prior_gpu.py tests/test_flamed_gpu.py -x -q -s --timeout 180 --timeout-method thread > gpurun_out/r03v/pytest.log 2>&1
grep -E "passed|failed|rel-L2" gpurun_out/r03v/pytest.log | tail -6
timeout -k 10 120 python tools/prior_profile.py bf16
