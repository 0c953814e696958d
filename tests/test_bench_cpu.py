"""bench.py's multi-rank launcher (BASELINE configs[3] scaling runs) rehearsed on CPU:
`--gpus 2` outside torchrun starts two ranks of bench.py as a child torch.distributed.run job (gloo in
--plumbing mode), rank 0 prints one JSON line whose n_gpus / global_batch describe the whole job."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, capture_output=True, text=True,
                       timeout=600, env=env, cwd=REPO)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


def test_launcher_world2():
    line = _run(["--gpus", "2", "--plumbing", "--steps", "1", "--warmup", "1", "--frames", "12", "--nfe", "2",
                 "--batch", "1"])
    assert line["n_gpus"] == 2
    assert line["config"]["global_batch"] == 2
    assert line["finite"] and line["value"] > 0
    assert abs(line["value"] - 2 * 12 / (line["ms_per_step"] / 1e3)) / line["value"] < 1e-2


def test_single_rank_plumbing():
    line = _run(["--plumbing", "--steps", "1", "--warmup", "1", "--frames", "8", "--nfe", "2"])
    assert line["n_gpus"] == 1 and line["config"]["global_batch"] == 1


def test_world_mismatch_rejected():
    env = {k: v for k, v in os.environ.items()}
    env.update({"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "4", "--plumbing"], capture_output=True,
                       text=True, timeout=300, env=env, cwd=REPO)
    assert p.returncode != 0 and "WORLD_SIZE=2" in (p.stderr + p.stdout)
