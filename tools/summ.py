"""One-line summary of bench.py JSON outputs: ms/solve, graph step us, per-class in-graph us."""
import json
import sys

for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    ks = " ".join(f"{k['name'][:10]}={k['us']}" for k in d["kernels"])
    print(f"{f}: ms/solve={d['ms_per_step']:.2f} step_us={d.get('step_us_graph')} | {ks}")
