#!/bin/bash
# GPU box: the whole -m gpu suite (one process, per-test timeout), then the round profile
# (tools/gpu_profile.sh: smoke, bench, rocprofv3 kernel stats, PMC passes).  Usage:
#   bash tools/gpu_suite.sh TAG [bench args]
set -u
TAG=${1:-r03}; shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread -rfEs > $OUT/pytest.log 2>&1
rc=$?
tail -5 $OUT/pytest.log
echo "pytest rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/gpu_profile.sh $TAG "$@"
