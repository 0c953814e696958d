#!/bin/bash
# GPU box, round 4: persistent tests; B = 1 A/B of the drain-behind-DMA order (persist_opt 4096);
# configs[2] A/B of the split-batch chains and the bf16 residual stream; the large-M parity tests.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r04h
mkdir -p $OUT
step() { "$@"; rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "step rc=$rc: stopping"; exit $rc; fi; return 0; }
bash tools/gpu_bench_ab.sh r04h 585 4681 1609 5705 16969 585 4681 5705 || exit $?
bash tools/gpu_b64_ab.sh r04h_b64 "--split-batch 1" "" "--split-batch 4" "--x16 1" || exit $?
step timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_configs_gpu.py -k "cfg2 or cfg4" > $OUT/cfg.log 2>&1
grep -E "passed|failed|rel-L2" $OUT/cfg.log | tail -20
