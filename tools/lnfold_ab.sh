# LayerNorm-fold A/B: fold error-budget test (prints both errors), then B=64 throughput solves with lnfold 0 / 1.
set -o pipefail
mkdir -p gpurun_out/lnfold
timeout -k 10 300 python -u -m pytest tests/test_denoiser_gpu.py -x -q -s -k "lnfold" --timeout 120 --timeout-method thread > gpurun_out/lnfold/err.log 2>&1; rc=$?; grep -E "rel-L2|passed|failed" gpurun_out/lnfold/err.log; [ $rc -eq 0 ] || exit $rc
for a in "--lnfold 0" "--lnfold 1"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --batch 64 --steps 3 --warmup 1 $a > gpurun_out/lnfold/b64_${a// /}.json 2>gpurun_out/lnfold/b64.err || exit 1
  echo "[$a] B=64"; python tools/summ.py gpurun_out/lnfold/b64_${a// /}.json
done
