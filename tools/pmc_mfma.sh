#!/bin/bash
# MFMA-side and traffic evidence per kernel class: a kernel-trace run and separate rocprofv3 --pmc
# passes (one counter group per pass, no trace domains with --pmc), each under its own time limit; the persistent
# kernels run as plain launches (--coop 0: rocprofv3's teardown faults after cooperative ones, README).  Then
# tools/pmc_summary.py writes OUT/summary.md + summary.json.  Usage: bash tools/pmc_mfma.sh TAG [bench args]
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
# heartbeat under gpurun_out/ (a long profiled run prints nothing until it ends)
( while true; do date >> $OUT/heartbeat; sleep 50; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
BENCH="python3 $ROOT/bench.py --no-cpu-baseline --no-secondary --no-peaks --coop 0 --steps 1 --warmup 1 --kernel-iters 2 $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- $BENCH > $OUT/kt.log 2>&1 || { echo "kernel trace failed"; tail -5 $OUT/kt.log; exit 1; }
i=0
for grp in "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F8 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1)); echo "pmc pass $i: $grp" >&2
  timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- $BENCH > $OUT/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 $ROOT/tools/pmc_summary.py $OUT
# keep the summaries and rocprofv3's per-kernel stats; the raw per-dispatch CSVs are large (gpurun returns <= 64 MiB)
cp $(find $OUT/kt -name "*kernel_stats.csv" | head -1) $OUT/kernel_stats.csv 2>/dev/null
rm -rf $OUT/kt $OUT/p1 $OUT/p2 $OUT/p3 $OUT/p4
