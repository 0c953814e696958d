"""Multi-GPU path rehearsed on CPU: metadata utterances length-bucketed over ranks
(contiguous buckets balanced by total length), prompts round-robin, no data-path collective, timing
records gathered once, per-rank seeds seed + rank with per-shard parity against the oracle; world_size
2 over gloo via torch.distributed.run."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from _common import PKG

sys.path.insert(0, PKG)
from flamed.utils.audio import write_wav  # noqa: E402
from flamed.utils.dist import bucket_bounds, bucket_shard, shard  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


def test_shard_partition():
    items = list(range(11))
    parts = [shard(items, r, 4) for r in range(4)]
    assert sorted(x for p in parts for x in p) == items
    assert max(map(len, parts)) - min(map(len, parts)) <= 1
    assert shard(items, 0, 1) == items
    with pytest.raises(ValueError):
        shard(items, 2, 2)


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_bucket_shard_balance(world):
    rng = np.random.default_rng(world)
    costs = [int(c) for c in rng.integers(20, 600, 37)]
    items = list(range(len(costs)))
    parts = [bucket_shard(items, costs, r, world) for r in range(world)]
    assert sorted(x for p in parts for x in p) == items
    sums = [sum(costs[i] for i in p) for p in parts]
    # contiguous in length order, and every bucket within one (largest) item of the mean
    flat = [costs[i] for p in parts for i in p]
    assert flat == sorted(costs)
    assert max(abs(s_ - sum(costs) / world) for s_ in sums) <= max(costs)
    assert all(parts)


def test_bucket_bounds_edges():
    assert bucket_bounds([], 3) == [(0, 0), (0, 0), (0, 0)]
    assert bucket_bounds([5, 5], 4) == [(0, 1), (1, 2), (2, 2), (2, 2)]
    assert bucket_bounds([1, 1, 1, 1], 2) == [(0, 2), (2, 4)]
    with pytest.raises(ValueError):
        bucket_shard([1], [1, 2], 0, 1)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("mode", ["metadata", "prompts"])
def test_two_rank_sharded_synthesis(tmp_path, mode):
    rng = np.random.default_rng(0)
    os.makedirs(tmp_path / "pr")
    for i in range(3):
        write_wav(str(tmp_path / "pr" / f"p{i}.wav"), rng.normal(0, 0.1, 4000).astype(np.float32))
    lines = [f"u{i}.wav|p{i % 3}.wav|utterance number {i}." for i in range(5)]
    (tmp_path / "meta.txt").write_text("\n".join(lines) + "\n")
    env = dict(os.environ, OMP_NUM_THREADS="2", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(HERE, "_dist_worker.py"),
           str(tmp_path), mode]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads((tmp_path / f"result_{mode}.json").read_text())
    locs = [json.loads((tmp_path / f"rank{k}_{mode}.json").read_text())["local"] for k in range(2)]
    n = 5 if mode == "metadata" else 3
    assert res["world"] == 2 and res["n_total"] == n and sum(locs) == n and min(locs) >= 1
    out = tmp_path / "out" / ("nfe2-temp0.3" if mode == "metadata" else "")
    files = sorted(os.listdir(out))
    if mode == "metadata":
        assert files == [f"u{i}.wav" for i in range(5)]
    else:
        assert files == [f"p{i}-2-2-0.3-0.3.wav" for i in range(3)]
    assert res["rtf"] > 0
    if mode == "metadata":
        ranks = [json.loads((tmp_path / f"rank{k}_{mode}.json").read_text()) for k in range(2)]
        costs = ranks[0]["costs"]
        assert sorted(ranks[0]["shard"] + ranks[1]["shard"]) == list(range(5))
        assert max(costs[i] for i in ranks[0]["shard"]) <= min(costs[i] for i in ranks[1]["shard"])  # buckets
        assert abs(ranks[0]["cost"] - ranks[1]["cost"]) <= max(costs)
        assert all(r["shard_rel_l2"] < 1e-5 for r in ranks)
