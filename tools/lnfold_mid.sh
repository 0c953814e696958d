# LayerNorm fold A/B across the large-M path's small end (B*T = 1600 .. 6400, and long-form T=2400 nfe=256).
set -o pipefail
mkdir -p gpurun_out/lnfmid
for cfg in "--batch 1 --frames 2400 --nfe 256" "--batch 4 --frames 400" "--batch 8 --frames 400" "--batch 16 --frames 400"; do
  for f in 0 1; do
    tag=$(echo "$cfg $f" | tr -d ' -')
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --steps 3 --warmup 1 $cfg --lnfold $f > gpurun_out/lnfmid/$tag.json 2>gpurun_out/lnfmid/err.log || exit 1
    echo "[$cfg lnfold $f]"; python tools/summ.py gpurun_out/lnfmid/$tag.json
  done
done
