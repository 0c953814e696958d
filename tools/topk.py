"""Top kernels of a rocprofv3 --stats run: python tools/topk.py <dir>/run_kernel_stats.csv [N]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[: int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
    name = r["Name"]
    print(f"{float(r['TotalDurationNs']) / 1e6:9.2f} ms {int(r['Calls']):6d} calls {float(r['AverageNs']) / 1e3:9.2f} us  {name[:160]}")
