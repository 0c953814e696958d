bash tools/gpu_steps.sh r06d \
 counters 120 "rocprofv3 -L > gpurun_out/r06d/counters_full.txt 2>&1; grep -i -o 'SQ_[A-Z0-9_]*MFMA[A-Z0-9_]*\|SQ_INSTS_[A-Z0-9_]*\|SQ_LDS[A-Z0-9_]*\|GRBM_[A-Z_]*\|TCC_EA0_[A-Z_]*' gpurun_out/r06d/counters_full.txt | sort -u" \
 persist 600 "python -u -m pytest tests/test_persist_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu" \
 configs 900 "python -u -m pytest tests/test_configs_gpu.py -x -v --timeout 300 --timeout-method thread -m gpu -k 'concurrent or split_batch'" \
 bench 400 "python -u bench.py --steps 20 --warmup 3 --no-secondary"
