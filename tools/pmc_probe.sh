# PMC counters of the GEMM probe kernels at M=25600 (one counter group per pass, no trace domains).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmcprobe
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 $R/tools/probe_gemm.py 25600 > $OUT/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 - $OUT <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{out}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "gemm" not in k:
            continue
        k = k.replace("_ZN2fl", "")[:60]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    m = {c: sum(v) / len(v) for c, v in d.items()}
    wc = m.get("SQ_WAVE_CYCLES", 0) or 1
    print(k)
    print("   " + "  ".join(f"{c}={v:.4g}" for c, v in sorted(m.items())))
    if "SQ_WAIT_ANY" in m:
        print(f"   wait_any={m['SQ_WAIT_ANY']/wc:.2f} wait_inst={m['SQ_WAIT_INST_ANY']/wc:.2f} active={m['SQ_ACTIVE_INST_ANY']/wc:.2f} "
              f"lds_conflict/idx={m['SQ_LDS_BANK_CONFLICT']/max(1,m['SQ_LDS_IDX_ACTIVE']):.3f}")
    if "TCC_HIT_sum" in m:
        print(f"   L2 hit rate={m['TCC_HIT_sum']/max(1,m['TCC_HIT_sum']+m['TCC_MISS_sum']):.3f}")
PY
