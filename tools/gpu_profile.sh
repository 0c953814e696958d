#!/bin/bash
# Round profile on the GPU box: smoke, bench (with CPU baseline), rocprofv3 kernel stats of the bench,
# and separate PMC passes for HBM traffic of the bench (profiled runs use plain launches of the persistent
# kernels, --coop 0: rocprofv3 faults at exit after cooperative ones, README).  Usage: bash tools/gpu_profile.sh TAG [bench args]
set -u
TAG=${1:-r01}; shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $ROOT
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
timeout -k 10 400 python3 bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $ROOT/bench.py --no-cpu-baseline --no-secondary --no-peaks --coop 0 --steps 2 --warmup 1 "$@" > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $ROOT/bench.py --no-cpu-baseline --no-secondary --no-peaks --coop 0 --steps 1 --warmup 1 "$@" > $OUT/pmc1.log 2>&1 || { echo "pmc fetch failed"; tail -20 $OUT/pmc1.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 $ROOT/bench.py --no-cpu-baseline --no-secondary --no-peaks --coop 0 --steps 1 --warmup 1 "$@" > $OUT/pmc2.log 2>&1 || { echo "pmc write failed"; tail -20 $OUT/pmc2.log; exit 1; }
echo "profile done"
cat $OUT/bench.json
