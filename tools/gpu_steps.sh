#!/bin/bash
# GPU box: run named steps in order, each under its own time limit, output in gpurun_out/TAG/NAME.log.  A step
# that exits 0 or 1 (test failures) lets the next one run; a time limit, abort, segfault or any other status
# ends the run there (nothing more touches the GPU after a fault).  Usage:
#   bash tools/gpu_steps.sh TAG NAME SECONDS 'COMMAND' [NAME SECONDS 'COMMAND' ...]
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $ROOT
while [ $# -ge 3 ]; do
  name=$1; secs=$2; cmd=$3; shift 3
  echo "== $name (limit ${secs}s): $cmd"
  timeout -k 10 $secs bash -c "$cmd" > $OUT/$name.log 2>&1
  rc=$?
  tail -4 $OUT/$name.log
  echo "== $name rc=$rc"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "stopping after $name (rc=$rc)"; exit $rc; }
done
