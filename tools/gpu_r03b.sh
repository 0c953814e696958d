set -u
mkdir -p gpurun_out/r03b
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_persist_gpu.py -v -s --timeout 180 --timeout-method thread > gpurun_out/r03b/persist.log 2>&1
rc=$?
echo "persist pytest rc=$rc" >> gpurun_out/r03b/persist.log
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 300 python -u -m pytest tests/test_denoiser_gpu.py tests/test_configs_gpu.py -q --timeout 180 --timeout-method thread -rfE > gpurun_out/r03b/den.log 2>&1
  echo "den pytest rc=$?" >> gpurun_out/r03b/den.log
fi
