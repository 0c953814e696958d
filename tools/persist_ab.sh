# A/B of the persistent kernel's experiment bits (flamed_tune persist_opt) at B = 1, T = 400, nfe = 128.
set -u
OUT=gpurun_out/${1:-pab}
mkdir -p $OUT
shift || true
for o in "$@"; do
  timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-secondary --no-cpu-baseline --no-peaks --persist-opt $o > $OUT/o$o.json 2> $OUT/o$o.err || exit 1
  python3 -c "import json; p = json.load(open('$OUT/o$o.json')); print('opt', $o, p['ms_per_step'])"
done
