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


def test_launcher_world2_configs3_labels():
    """a multi-rank run is labelled as the configs[3] layout with its global batch, every
    rank's own frames/s and the efficiency against rank 0 running the same per-GPU workload alone."""
    line = _run(["--gpus", "2", "--plumbing", "--config", "3", "--batch", "4", "--frames", "12", "--nfe", "2",
                 "--steps", "1", "--warmup", "1"])
    cfg = line["config"]
    assert "configs[3]" in cfg["workload"] and "utterance-sharded over 2 GPU" in cfg["workload"], cfg["workload"]
    assert cfg["global_batch"] == 8 and cfg["batch_per_gpu"] == 4
    per = line["per_rank_frames_per_s"]
    assert len(per) == 2 and all(v > 0 for v in per)
    eff = line["scaling_detail"]
    assert eff["solo_rank0_frames_per_s"] > 0 and 0.0 < eff["efficiency_vs_n1"] < 4.0
    assert abs(line["value"] - 2 * 4 * 12 / (line["ms_per_step"] / 1e3)) / line["value"] < 1e-2


def test_single_rank_labels():
    """One rank: B = 1 is labelled configs[1]; --config 2 at a reduced size names configs[2] and says so."""
    one = _run(["--plumbing", "--steps", "1", "--warmup", "1", "--frames", "8", "--nfe", "2"])
    assert "configs[1]" in one["config"]["workload"] and one["scaling_detail"] is None
    two = _run(["--plumbing", "--config", "2", "--batch", "2", "--frames", "8", "--nfe", "2", "--steps", "1", "--warmup", "1"])
    assert "configs[2]" in two["config"]["workload"] and "non-reference size" in two["config"]["workload"]
    assert two["config"]["global_batch"] == 2
