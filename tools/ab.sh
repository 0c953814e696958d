# Generic bench A/B: tools/ab.sh TAG "args A" "args B" ... ; B=1 at T=400 and T=131, after the denoiser parity tests.
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest tests/test_denoiser_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1; rc=$?; tail -2 gpurun_out/$TAG/tests.log
[ $rc -eq 0 ] || exit $rc
i=0
for a in "$@"; do
  i=$((i+1))
  for T in 400 131; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --frames $T $a > gpurun_out/$TAG/v${i}_T$T.json 2>gpurun_out/$TAG/v${i}_T$T.err || exit 1
    echo "[$a] T=$T"; python tools/summ.py gpurun_out/$TAG/v${i}_T$T.json
  done
done
