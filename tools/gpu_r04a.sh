#!/bin/bash
# GPU box, round 4: persistent-solve contract tests, new parity tests, persist_opt A/B with timelines.
# A step that crashes, faults or times out (any status other than 0 or pytest's 1 = tests failed) ends the run.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r04a
mkdir -p $OUT
step() { "$@"; rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "step rc=$rc: stopping"; exit $rc; fi; return 0; }
step timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_persist_gpu.py > $OUT/persist.log 2>&1
tail -5 $OUT/persist.log
step timeout -k 10 500 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread tests/test_configs_gpu.py::test_cfg4_bf16_solve_256_vs_oracle tests/test_flamed_gpu.py::test_end_to_end_duration_flips_vs_oracle > $OUT/parity.log 2>&1
tail -3 $OUT/parity.log
bash tools/gpu_ab.sh r04a_ab 585 1609 2633 3657
