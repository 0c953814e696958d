"""bench.py's multi-rank GPU branch on the one GPU a test box has: `--dist-single` runs the
branch a driver scaling run takes at N > 1 -- an RCCL ("nccl") process group, the device-tensor max-over-ranks
all-reduces of scaling_stats and the configs[3] leg (64 utterances x 400 frames per GPU) -- as a group of one
rank, so that code has executed on hardware before an 8-GPU job depends on it."""
import json
import os
import subprocess
import sys

import pytest

from _common import PKG

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(PKG)


def test_bench_single_rank_dist_branch():
    args = ["--dist-single", "--steps", "1", "--warmup", "1", "--no-secondary", "--no-cpu-baseline", "--no-peaks",
            "--kernel-iters", "2"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, capture_output=True, text=True,
                       cwd=REPO, env=env, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 1 and line["finite"]
    assert len(line["per_rank_frames_per_s"]) == 1
    eff = line["scaling_detail"]
    assert eff is not None and 0.5 < eff["efficiency_vs_n1"] < 1.5, eff
    c3 = line["configs3"]
    assert c3 is not None and c3["global_batch"] == 64 and "BASELINE configs[3]" in c3["workload"]
    assert c3["value"] > 0 and len(c3["per_rank_frames_per_s"]) == 1 and c3["scaling_detail"]["efficiency_vs_n1"] > 0.5
    print("single-rank dist branch:", line["value"], "frames/s; configs[3] leg", c3["value"], "frames/s, efficiency",
          eff["efficiency_vs_n1"], c3["scaling_detail"]["efficiency_vs_n1"])
