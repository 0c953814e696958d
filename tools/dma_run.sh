# A/B of the GEMM main loops (flamed_tune dma 0/1/2): parity tests, bench B=1/B=8 with in-graph per-class costs.
set -o pipefail
mkdir -p gpurun_out/dma
timeout -k 10 300 python -u -m pytest tests/test_denoiser_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dma/tests.log 2>&1; rc=$?; tail -3 gpurun_out/dma/tests.log
[ $rc -eq 0 ] || exit $rc
for d in ${DMAS:-1 0 2}; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --dma $d > gpurun_out/dma/b1_$d.json 2>gpurun_out/dma/b1_$d.err || exit 1
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --dma $d --batch 8 --steps 3 > gpurun_out/dma/b8_$d.json 2>gpurun_out/dma/b8_$d.err || exit 1
done
for f in gpurun_out/dma/b*.json; do python -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['ms_per_step'], d.get('step_us_graph'), ' '.join(f\"{k['name'][:10]}={k['us']}\" for k in d['kernels']))"; done
